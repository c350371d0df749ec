"""Checkpoint / metrics formats: what the trainer writes is what the
reference's consumers read.

* checkpoint_{tag}.pt holds the reference's keys (trainer.py:231-245) and loads with torch's safe
  default loader, the scripts/evaluate.py:271-279 way: rebuild the model from
  checkpoint["config"]["model"] through the registry, then load_state_dict.
* load_checkpoint restores epoch, step, best loss, optimizer and scheduler state.
* metrics.json: train_/val_ prefixed lists per epoch (trainer.py:166-184, 325-330).
* FusedAdam's state_dict loads into torch.optim.Adam and back, and the next steps agree (GPU)."""
import json
import logging
import tempfile
from pathlib import Path

import pytest
import torch

from src.models import model_registry
from src.training.trainer import ContrastiveTrainer

CKPT_KEYS = {"epoch", "global_step", "model_state_dict", "optimizer_state_dict", "scheduler_state_dict",
             "best_val_loss", "config"}


class _Loader:
    class dataset:  # noqa: N801
        @staticmethod
        def __len__():
            return 0


def _trainer(model, opt, sched, cfg, out):
    return ContrastiveTrainer(model, _Loader(), None, None, opt, sched, torch.device("cpu"), cfg, out,
                              logging.getLogger("ckpt"))


@pytest.mark.parametrize("mtype", ["phoneme_cnn", "phoneme_cnn_deep"])
def test_checkpoint_loads_the_evaluate_way(mtype):
    cfg = {"model": {"type": mtype, "embedding_dim": 64, "use_attention": True}, "training": {"epochs": 3}}
    torch.manual_seed(3)
    m = model_registry.create(mtype, cfg["model"])
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-4)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=3)
    # give the optimizer real state (a CPU step with synthetic gradients; no kernel runs)
    for p in m.parameters():
        p.grad = torch.randn_like(p)
    opt.step()
    sched.step()
    out = Path(tempfile.mkdtemp())
    t = _trainer(m, opt, sched, cfg, out)
    t.current_epoch, t.global_step, t.best_val_loss = 2, 17, 0.625
    t._save_checkpoint("best")

    path = out / "checkpoints" / "checkpoint_best.pt"
    ck = torch.load(path, map_location="cpu")  # torch's default: weights_only=True
    assert set(ck) == CKPT_KEYS
    assert ck["epoch"] == 2 and ck["global_step"] == 17 and ck["best_val_loss"] == 0.625
    m2 = model_registry.create(ck["config"]["model"]["type"], ck["config"]["model"])
    m2.load_state_dict(ck["model_state_dict"])  # strict
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k]), k

    # resume into a fresh trainer
    m3 = model_registry.create(mtype, cfg["model"])
    opt3 = torch.optim.Adam(m3.parameters(), lr=1e-3, weight_decay=1e-4)
    sched3 = torch.optim.lr_scheduler.CosineAnnealingLR(opt3, T_max=3)
    t3 = _trainer(m3, opt3, sched3, cfg, out)
    t3.load_checkpoint(path)
    assert (t3.current_epoch, t3.global_step, t3.best_val_loss) == (2, 17, 0.625)
    assert sched3.last_epoch == 1 and opt3.param_groups[0]["lr"] == opt.param_groups[0]["lr"]
    for p, q in zip(m.parameters(), m3.parameters()):
        assert torch.equal(opt.state[p]["exp_avg"], opt3.state[q]["exp_avg"])
        assert torch.equal(opt.state[p]["exp_avg_sq"], opt3.state[q]["exp_avg_sq"])


def test_metrics_json_layout():
    m = torch.nn.Linear(2, 2)
    opt = torch.optim.SGD(m.parameters(), 0.1)
    out = Path(tempfile.mkdtemp())
    t = _trainer(m, opt, None, {}, out)
    t._log_metrics({"loss": 1.5, "lr": 0.001}, {"loss": 1.25, "linear_accuracy": 0.5, "rf_accuracy": 0.25})
    t.current_epoch = 1
    t._log_metrics({"loss": 1.0, "lr": 0.0005}, {})
    t._save_metrics()
    got = json.loads((out / "metrics.json").read_text())
    assert got == {"train_loss": [1.5, 1.0], "train_lr": [0.001, 0.0005], "val_loss": [1.25],
                   "val_linear_accuracy": [0.5], "val_rf_accuracy": [0.25]}


def test_perf_json_layout():
    """perf.json: one record per epoch with samples/s and the step's roofline
    fractions from phoneme_contrast_amd.costs (cnn_small at B = 4096, T = 200: 3.27 TFLOP executed, 7.29
    TFLOP direct-conv equivalent, 73.7 GB)."""
    m = model_registry.create("phoneme_cnn", {"embedding_dim": 128})
    out = Path(tempfile.mkdtemp())
    t = _trainer(m, torch.optim.SGD(m.parameters(), 0.1), None, {}, out)
    t._record_perf(10, 40960, 0.5, (4096, 1, 40, 200))
    t.current_epoch = 1
    t._record_perf(0, 0, 0.0, None)
    t._save_metrics()
    got = json.loads((out / "perf.json").read_text())
    e0 = got["epochs"][0]
    assert got["world_size"] == 1 and len(got["epochs"]) == 2 and got["epochs"][1]["steps"] == 0
    assert e0["ms_per_step"] == 50.0 and e0["samples_per_s"] == 81920.0
    # executed FLOPs: the Winograd convs of layers 2-6 at 4/9 of their direct-conv count
    assert abs(e0["step_tflops"] - 3267966795776 / 0.05 / 1e12) < 0.01
    assert e0["schema"] == 2
    assert abs(e0["executed_mfma_fraction"] - 3267966795776 / 0.05 / 157.3e12) < 1e-4
    assert abs(e0["mfma_fraction"] - 7294498635776 / 0.05 / 157.3e12) < 1e-4
    assert 0 < e0["hbm_fraction"] < 1


@pytest.mark.gpu
def test_fused_adam_state_interchanges_with_torch_adam():
    """Checkpoint written with FusedAdam (GPU, one flat buffer) -> torch.optim.Adam on CPU: the
    moments and step carry over and the next update agrees; and back again."""
    from phoneme_contrast_amd.optim import FusedAdam
    torch.manual_seed(5)
    m = model_registry.create("phoneme_cnn", {"embedding_dim": 64}).cuda()
    opt = FusedAdam(m.parameters(), lr=1e-3, weight_decay=1e-4)
    grads = [[torch.randn_like(p) for p in m.parameters()] for _ in range(3)]
    for gs in grads[:2]:
        for p, g in zip(m.parameters(), gs):
            p.grad = g.clone()
        opt.step()
    out = Path(tempfile.mkdtemp())
    torch.save({"model_state_dict": m.state_dict(), "optimizer_state_dict": opt.state_dict()}, out / "c.pt")
    ck = torch.load(out / "c.pt", map_location="cpu")

    mc = model_registry.create("phoneme_cnn", {"embedding_dim": 64})
    mc.load_state_dict(ck["model_state_dict"])
    oc = torch.optim.Adam(mc.parameters(), lr=1e-3, weight_decay=1e-4)
    oc.load_state_dict(ck["optimizer_state_dict"])
    for p, q in zip(m.parameters(), mc.parameters()):
        assert int(oc.state[q]["step"]) == 2
        assert torch.equal(opt.state[p]["exp_avg"].cpu(), oc.state[q]["exp_avg"])
    for (p, q), g in zip(zip(m.parameters(), mc.parameters()), grads[2]):
        p.grad, q.grad = g.clone(), g.cpu()
    opt.step()
    oc.step()
    for p, q in zip(m.parameters(), mc.parameters()):
        assert torch.allclose(p.detach().cpu(), q.detach(), rtol=0, atol=1e-6)

    # torch.optim.Adam state -> a fresh FusedAdam on the GPU
    mg = model_registry.create("phoneme_cnn", {"embedding_dim": 64}).cuda()
    mg.load_state_dict(mc.state_dict())
    og = FusedAdam(mg.parameters(), lr=1e-3, weight_decay=1e-4)
    og.load_state_dict(oc.state_dict())
    gs = [torch.randn_like(q) for q in mc.parameters()]
    for p, q, g in zip(mg.parameters(), mc.parameters(), gs):
        p.grad, q.grad = g.cuda(), g.clone()
    og.step()
    oc.step()
    for p, q in zip(mg.parameters(), mc.parameters()):
        assert torch.allclose(p.detach().cpu(), q.detach(), rtol=0, atol=1e-6)
