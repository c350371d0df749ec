"""Cross-check of the Winograd F(2x2,3x3) conv's fused epilogues (csrc/conv_wino.hip) against the
direct LDS-DMA conv (csrc/conv_dma.hip) on the same operands, at the cnn_small layer shapes:
forward with the producer's BN+ReLU prologue and the BN (sum, M2) partials, the data gradient
through ReLU + BN-backward sums, through MaxPool2 + Dropout2d (16-byte and scalar window paths; and from the selection the
forward's pool recorded, EPI_BWD_POOLSEL),
and plain store.  tools/wino_bench (built by `make`) runs both engines and exits 2 when the outputs
differ by more than 1e-5 of max|out| or the per-channel partial sums by more than 1e-4 (fp32
rounding of two exact-arithmetic conv algorithms).  The direct engine is pinned to the reference by
the model golden tests (tests/test_model_gpu.py, T = 50 routes through it); the Winograd engine is
also checked against float64 torch in tests/test_conv2d_gpu.py."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "tools", "wino_bench")

CASES = [  # H, W, cin, cout, B, reps, epilogue, prologue
    (40, 200, 32, 32, 48, 1, 0, 1),    # L2 forward: BN+ReLU prologue, statistics epilogue
    (20, 100, 32, 64, 48, 1, 0, 0),    # L3 forward on the materialised pooled input
    (40, 200, 32, 32, 48, 1, 1, 0),    # L2 data gradient through ReLU
    (20, 100, 64, 32, 48, 1, 2, 0),    # L3 data gradient through MaxPool2 (16-byte windows)
    (10, 50, 128, 64, 48, 1, 2, 0),    # L5 data gradient through MaxPool2
    (20, 100, 64, 32, 48, 1, 4, 0),    # L3 through MaxPool2 from the forward's recorded selection
    (10, 50, 128, 64, 48, 1, 4, 0),    # L5 likewise
    (20, 101, 64, 32, 24, 1, 4, 0),    # odd pooled width: scalar windows and stores
    (40, 201, 32, 32, 24, 1, 0, 1),    # T = 201: odd width, scalar stores
    (40, 201, 32, 32, 24, 1, 1, 0),
    (20, 100, 64, 64, 24, 1, 3, 0),    # plain store (cnn_deep's stride-1 data gradients)
    # narrow images on batch-spanning units (cnn_deep blocks 3 / 4 at T = 200 / 201): a wave's 16 tiles in
    # up to 4 row segments of several samples; odd batches end inside a unit
    (5, 25, 256, 256, 24, 1, 0, 0),
    (5, 25, 256, 256, 23, 1, 3, 0),
    (3, 13, 512, 512, 16, 1, 0, 0),
    (3, 13, 512, 512, 17, 1, 3, 0),
    (5, 26, 64, 128, 9, 1, 0, 0),
    (4, 14, 32, 64, 5, 1, 3, 0),
    (1, 30, 32, 32, 3, 1, 0, 0),
]


@pytest.mark.parametrize("queue", [0, 1])
@pytest.mark.parametrize("case", CASES)
def test_winograd_epilogues_match_direct_engine(case, queue):
    """queue = 1: units taken from the per-XCD work queue (ConvArgs::queue); wino_bench launches the
    kernel several times on one queue, checks the last launch's output and that the queue is left zero."""
    assert os.path.exists(BENCH), "tools/wino_bench missing: run make"
    env = dict(os.environ, WINO_QUEUE=str(queue))
    r = subprocess.run([BENCH] + [str(v) for v in case], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, (case, r.stdout, r.stderr)
    assert ("(queue)" in r.stdout) == bool(queue), r.stdout


WB = os.path.join(ROOT, "tools", "wb_bench")
WB_CASES = [  # H, W, B, reps [, pooled dz]: the fused layer-2 backward (wgbd_wino) vs wgrad_wino + conv_wino's data gradient
    (40, 200, 48, 1),   # cnn_small T = 200: strips of 48 + 52 tiles
    (20, 100, 24, 1),   # T = 100: one 50-tile strip (4 data-gradient groups, the last partial)
    (21, 56, 16, 1),    # odd H (a half tile row at the bottom), one 28-tile strip
    (40, 200, 48, 1, 1),  # dz as layer 3's pooled gradient + window selection (EPI_BWD_POOLSELP's output)
    (20, 100, 24, 1, 1),
    (40, 200, 16, 1, 1, 1),  # producer BN scale 0 / tiny on three channels: xhat from yp itself
    (20, 100, 8, 1, 0, 1),
]


@pytest.mark.parametrize("case", WB_CASES)
def test_fused_layer2_backward_matches_two_kernel_path(case):
    """dW, dz_prev and the producer BN's backward sums of the one-pass kernel agree with the two
    kernels it replaces (both Winograd, fp32: rounding-level differences only, <= 2e-5 relative)."""
    assert os.path.exists(WB), "tools/wb_bench missing: run make"
    r = subprocess.run([WB] + [str(v) for v in case], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, (case, r.stdout, r.stderr)


WW = os.path.join(ROOT, "tools", "ww_bench")
WW_CASES = [  # H, W, cin, cout, B, reps, prologue, pooled dz
    (20, 100, 64, 64, 48, 1, 1, 1),  # cnn_small layer 4 behind layer 5's pool: dz rebuilt from the selection
    (20, 100, 64, 64, 48, 1, 1, 0),
    # odd widths (single-float staging, round 5) against the 32x32 row-window kernel: cnn_deep block 3 at
    # T = 200, an odd batch with the BN + ReLU prologue, a 7-row image (4 tile rows)
    (5, 25, 256, 256, 24, 1, 0, 0),
    (5, 25, 64, 96, 23, 1, 1, 0),
    (7, 27, 32, 32, 5, 1, 1, 0),
    (9, 29, 32, 32, 7, 1, 1, 0),  # the widest single-float image the staging capacity admits (15 tile columns)
    # cnn_small layers 6 / 5 (V = 2) with several tasks per slice: each task's prologue is loaded during the
    # previous task's last tile row (round 6)
    (10, 50, 128, 128, 100, 1, 1, 0),
    (10, 50, 64, 128, 200, 1, 0, 0),
    (11, 50, 64, 64, 300, 1, 1, 0),  # odd H: a half last tile row
]


@pytest.mark.parametrize("case", WW_CASES)
def test_winograd_wgrad_pooled_dz_matches_pixel_stream(case):
    """wgrad_wino reading dz as a pooled gradient + window selection (EPI_BWD_POOLSELP's output), or at odd
    widths, against the pixel-stream (narrow rows: row-window) weight gradient on the same dz (dW within 1e-4,
    dy exact)."""
    assert os.path.exists(WW), "tools/ww_bench missing: run make"
    r = subprocess.run([WW] + [str(v) for v in case], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, (case, r.stdout, r.stderr)


WS = os.path.join(ROOT, "tools", "ws_bench")
WS_CASES = [  # H, W, cin, cout, B, reps, prologue: the 32x32 row-window weight gradient (cnn_deep's narrow
    # blocks) vs the pixel-stream kernel; a slice's tasks stream their rows across task ends
    (3, 13, 512, 512, 24, 1, 0),
    (5, 25, 256, 256, 23, 1, 0),
    (5, 26, 256, 256, 9, 1, 1),
    (1, 30, 64, 64, 7, 1, 1),
    (10, 50, 128, 128, 5, 1, 0),
]


@pytest.mark.parametrize("case", WS_CASES)
def test_row_window_wgrad_matches_pixel_stream(case):
    assert os.path.exists(WS), "tools/ws_bench missing: run make"
    r = subprocess.run([WS] + [str(v) for v in case], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (case, r.stdout, r.stderr)
    assert " w32: " in r.stdout, r.stdout
