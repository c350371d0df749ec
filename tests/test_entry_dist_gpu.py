"""The N > 1 entry points the driver's scaling run executes, run as fresh processes on the one GPU.

* `bench.py --gpus 2` under `python -m torch.distributed.run --nproc-per-node 2` (exactly the
  driver's launch line) with PCX_DIST_BACKEND=gloo (two RCCL ranks cannot share one device), plain
  and `--global-supcon`: one JSON line from rank 0 with n_gpus 2, global_batch 2 x per-GPU, several
  all-reduce buckets, a finite loss and value > 0.
* The RCCL backend itself: `bench.py` under the launcher at world size 1 with PCX_DIST_FORCE_INIT=1
  (backend "nccl" = RCCL, eager init with device_id, bucket all-reduces on the side stream behind
  the native backward, FusedAdam on the bucketer's buffer) gives the same final loss as the plain
  single-process bench.
* `scripts/train.py main()` under the launcher at world size 2 for one synthetic epoch: both ranks end
  with bit-identical parameters and buffers (rank-0 broadcast, summed gradients, identical Adam),
  with FusedAdam (bucketed all-reduce) and with torch.optim.Adam (no bucketer attached,
  the trainer's flat all-reduce into p.grad); the two optimizers' runs follow the same trajectory.
* `scripts/train.py main()` on a WAV tree (accel.synthetic_data=false): parse_dataset ->
  WaveformStore.from_files -> sampler -> GPU views -> one epoch.
"""
import json
import os
import socket
import subprocess
import sys
import tempfile
import wave
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _launch(nproc, script_args, extra_env=None, timeout=300):
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.update(extra_env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}"] + script_args
    p = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=timeout)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-6000:])
    return p.stdout, p.stderr


def _bench_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


BENCH = ["bench.py", "--steps", "3", "--warmup", "1", "--batch", "512", "--no-cpu-baseline", "--no-peaks"]


@pytest.mark.parametrize("global_supcon", [False, True])
def test_bench_two_ranks_under_the_launcher(global_supcon):
    args = BENCH[:1] + ["--gpus", "2"] + BENCH[1:] + (["--global-supcon"] if global_supcon else [])
    out, err = _launch(2, args, {"PCX_DIST_BACKEND": "gloo"})
    d = _bench_line(out)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 1024 and d["config"]["per_gpu_batch"] == 512
    assert d["config"]["parallelism"] == "dp2" and d["config"]["dist_backend"] == "gloo"
    assert d["config"]["allreduce_buckets"] > 1
    assert np.isfinite(d["final_loss"]) and d["value"] > 0 and d["ms_per_step"] > 0
    assert ("global batch" in d["config"]["supcon"]) == global_supcon
    assert abs(d["value"] - 2 * 512 * 1000.0 / d["ms_per_step"]) <= 1e-3 * d["value"]
    assert d["roofline"] is not None and d["roofline"]["frac"] > 0


def test_bench_rccl_world1_matches_single_process():
    plain = json.loads([ln for ln in subprocess.run(
        [sys.executable] + BENCH + ["--no-kernel-timing"], cwd=ROOT, stdout=subprocess.PIPE,
        stderr=subprocess.PIPE, text=True, timeout=300, check=True).stdout.splitlines() if ln.startswith("{")][0])
    out, err = _launch(1, BENCH + ["--no-kernel-timing"], {"PCX_DIST_FORCE_INIT": "1"})
    d = _bench_line(out)
    assert d["config"]["dist_backend"] == "rccl" and d["config"]["allreduce_buckets"] > 1
    assert d["n_gpus"] == 1 and plain["config"]["allreduce_buckets"] == 0
    assert d["final_loss"] == plain["final_loss"], (d["final_loss"], plain["final_loss"])


SYN = ["accel.synthetic_data=true", "accel.synthetic.num_classes=64", "accel.synthetic.samples_per_class=3",
       "data.contrastive.classes_per_batch=8", "training.epochs=1", "training.batch_size=64", "model=cnn_small"]


def _train_two_ranks(extra):
    out = Path(tempfile.mkdtemp())
    _launch(2, [os.path.join("tests", "dist_train_worker.py"), str(out)] + SYN + extra, {"PCX_DIST_BACKEND": "gloo"},
            timeout=400)
    return [dict(np.load(out / f"rank{r}.npz")) for r in range(2)]


def test_train_entry_two_ranks_bit_identical():
    fused = _train_two_ranks([])
    torch_adam = _train_two_ranks(["accel.fused_adam=false"])
    for r0, r1 in (fused, torch_adam):
        keys = [k for k in r0 if k.startswith("p/")]
        assert len(keys) > 30
        for k in keys:
            assert np.array_equal(r0[k], r1[k]), k
        assert r0["global_step"][0] == r1["global_step"][0] >= 2
        assert np.isfinite(r0["train_loss"]).all()
    assert fused[0]["bucketer"][0] and not torch_adam[0]["bucketer"][0]
    # same data, same math: the two optimizers' runs follow the same trajectory (Adam normalises
    # each element's step to ~lr, so parameters agree to a few lr-sized steps, losses closely)
    steps = int(fused[0]["global_step"][0])
    for k in (k for k in fused[0] if k.startswith("p/") and "running" not in k and fused[0][k].dtype.kind == "f"):
        a, b = fused[0][k].astype(np.float64), torch_adam[0][k].astype(np.float64)
        assert np.abs(a - b).max() <= 2 * 3e-4 * steps, k
    assert np.allclose(fused[0]["train_loss"], torch_adam[0]["train_loss"], rtol=1e-3, atol=1e-4)


def _wav(path, n, sr, rng):
    path.parent.mkdir(parents=True, exist_ok=True)
    t = np.arange(n) / sr
    x = 0.3 * np.sin(2 * np.pi * rng.uniform(100, 2000) * t) + 0.02 * rng.standard_normal(n)
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(np.clip(np.round(x * 32767), -32768, 32767).astype("<i2").tobytes())


def test_train_entry_on_a_wav_tree():
    import importlib.util

    from phoneme_contrast_amd import config as cfglib
    rng = np.random.default_rng(3)
    root = Path(tempfile.mkdtemp()) / "New Stimuli 9-8-2024"
    names = ["ba", "da", "ga", "pa", "ta", "ka", "aba", "ada"]
    for i, nm in enumerate(names):
        for j in range(4):
            sub = ("CV", "Male" if j % 2 else "Female", "_a_") if len(nm) == 2 else ("VCV", "Female")
            sec = [1.2, 2.0, 2.6, 1.7][j]
            _wav(root.joinpath(*sub) / f"{nm}{j if j else ''}.wav", int(16000 * sec), 16000, rng)
    out = Path(tempfile.mkdtemp())
    cfg = cfglib.compose(os.path.join(ROOT, "configs"), "config",
                         [f"data.data_path={root}", "accel.synthetic_data=false", "training.epochs=1",
                          "data.contrastive.classes_per_batch=4", "training.batch_size=8", "model=cnn_small"],
                         output_dir=str(out))
    spec = importlib.util.spec_from_file_location("pcx_train_entry", os.path.join(ROOT, "scripts", "train.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    tr = mod.main(cfg)
    m = json.load(open(out / "metrics.json"))
    assert len(m["train_loss"]) == 1 and np.isfinite(m["train_loss"]).all() and np.isfinite(m["val_loss"]).all()
    assert tr.global_step == len(tr.train_loader) >= 1
    b = next(iter(tr.train_loader))
    assert tuple(b["views"].shape[1:]) == (2, 1, 40, 201)
    assert tr.train_loader.store.waves is not None  # < 500 files: the reference's cached crop
    assert (out / "checkpoints" / "checkpoint_final.pt").exists()
