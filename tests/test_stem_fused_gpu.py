"""Cross-check of the fused bf16 stem (csrc/conv.hip: stem_pool_kernel, stem_pool_bwd_kernel,
stem_wgrad_rc_kernel -- y0 recomputed, never stored) against the plane kernels that keep y0
(stem_fwd_mfma_kernel with its y0 output, maxpool3_fwd / maxpool3_bwd_prep, stem_wgrad_mfma_kernel)
on the same operands.  tools/stem_bench (built by `make`) exits 3 on any mismatch:
  * bitwise: BN0 statistics partials, the first-max taps (pooled NHWC), y0 at the selected taps,
    a0 = relu(BN0(y0 at the tap)), block 0's NHWC bf16 image, dz0 (== bf16 of the float path's g);
  * BN0 backward sums within 1e-5 (the per-window regrouping of the same sums);
  * the stem weight gradient within 2e-2 relative (dz0 rounded to bf16; measured 6e-4 at T = 200).
The plane kernels are pinned to the reference by the cnn_deep model tests (tests/test_deep_bf16_gpu.py
routes reduced-width stems through them).  Shapes: the T = 200 stem at B = 64, an odd-height / narrow
case, W % 4 != 0, and the widest supported row (W = 256)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "tools", "stem_bench")

CASES = [  # B, H, W, reps
    (64, 40, 200, 1),
    (37, 9, 30, 1),
    (5, 13, 57, 1),
    (3, 40, 256, 1),
    (8, 40, 201, 1),
]


@pytest.mark.parametrize("case", CASES)
def test_fused_stem_matches_plane_kernels(case):
    assert os.path.exists(BENCH), "tools/stem_bench missing: run make"
    r = subprocess.run([BENCH] + [str(v) for v in case], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (case, r.stdout, r.stderr)
