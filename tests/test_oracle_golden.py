"""Pin the CPU oracle (oracle/np_*.py, oracle/torch_port.py) against the reference's own outputs.

The fixtures were produced by importing the reference (tests/golden/make_golden.py); these
tests run on CPU only.  Tolerances:
  * float64 oracle vs the reference re-run in float64 (f64/*): tight (storage rounding only).
  * float64 oracle vs the reference's float32 run: loss <= 1e-4 (BASELINE contract),
    embeddings <= 1e-5; float32 gradients can legitimately differ where a ReLU/max-pool
    kink flips, so gradients are pinned by the f64 run instead.
"""
import numpy as np
import pytest

from golden_util import grad_errors, load, model_case
from oracle import np_models as nm
from oracle import np_ops as op

SUPCON_CASES = sorted({k.split("/")[0] for k in load("supcon").files})
MODEL_CASES = ["cnn_small_T200", "cnn_small_T201", "cnn_small_noattn_d64",
               "cnn_deep_T200", "cnn_deep_T201"]


@pytest.mark.parametrize("case", SUPCON_CASES)
def test_supcon_oracle_matches_reference(case):
    d = load("supcon")
    B, D, T, bT = d[case + "/meta"]
    mask = d[case + "/mask"] if case + "/mask" in d.files else None
    f = d[case + "/features"]
    if str(d[case + "/kind"]) == "supcon":
        loss, g = op.supcon_fwd_bwd(f, d[case + "/labels"], mask, T, bT, str(d[case + "/reduction"]))
    else:
        loss, g = op.ntxent_fwd_bwd(f, d[case + "/labels"], T, str(d[case + "/reduction"]))
    ref_loss = d[case + "/loss"]
    assert np.allclose(np.atleast_1d(loss), ref_loss, rtol=2e-6, atol=2e-6)
    ref_g = d[case + "/grad"]
    assert np.abs(g - ref_g).max() <= 2e-5 * np.abs(ref_g).max() + 2e-7


def test_supcon_oracle_errors():
    f = np.ones((1, 4)) / 2
    with pytest.raises(ValueError, match="Batch size must be greater than 1"):
        op.supcon_fwd_bwd(f, np.array([0]))
    with pytest.raises(ValueError):
        op.ntxent_fwd_bwd(np.ones((7, 4)), None)
    with pytest.raises(NotImplementedError):
        op.ntxent_fwd_bwd(np.ones((8, 4)), None)


@pytest.mark.parametrize("name", MODEL_CASES)
def test_model_oracle_matches_reference(name):
    c = model_case(name)
    e, loss, grads, new, opt = nm.train_step(c["state0"], c["x"], c["labels"],
                                             c["steps"][0]["masks"], c["temperature"], 0.07,
                                             c["lr"], c["weight_decay"])
    # float64 truth from the reference itself
    assert np.abs(e - c["f64"]["emb"]).max() < 1e-6
    assert abs(loss - c["f64"]["loss"]) < 1e-8
    for k, (kind, err) in grad_errors(grads, c["f64"]["grads"]).items():
        assert err < (1e-5 if kind == "rel" else 1e-6), (k, kind, err)
    # float32 reference run: the BASELINE loss contract and embeddings
    assert abs(loss - c["steps"][0]["loss"]) < 1e-4
    assert np.abs(e - c["steps"][0]["emb"]).max() < 1e-5


@pytest.mark.parametrize("name", ["cnn_small_T200", "cnn_deep_T200"])
def test_two_adam_steps_track_reference(name):
    """Two full train steps (forward, SupCon, backward, Adam) against the reference's state.
    Adam's first steps normalise each gradient element (update ~ lr*sign(g)), so elements
    whose gradient sits at float32 noise level may move by up to 2*lr differently; the bulk
    must agree tightly and the running statistics exactly."""
    c = model_case(name)
    _, l0, _, s1, opt = nm.train_step(c["state0"], c["x"], c["labels"], c["steps"][0]["masks"],
                                      c["temperature"], 0.07, c["lr"], c["weight_decay"])
    e1, l1, _, s2, _ = nm.train_step(s1, c["x"], c["labels"], c["steps"][1]["masks"],
                                     c["temperature"], 0.07, c["lr"], c["weight_decay"], opt)
    assert abs(l1 - c["steps"][1]["loss"]) < 2e-3
    lr = c["lr"]
    for k, ref in c["state_final"].items():
        got = np.asarray(s2[k], dtype=np.float64)
        if k.endswith("num_batches_tracked"):
            assert int(got) == int(ref) == 2
            continue
        diff = np.abs(got - ref)
        if k.endswith("running_mean") or k.endswith("running_var"):
            assert diff.max() < 1e-3 * max(1.0, np.abs(ref).max()), k
        else:
            assert diff.max() <= 4 * lr + 1e-5, k


def test_adam_oracle_matches_torch_adam():
    import torch
    g = np.random.default_rng(0)
    p0 = g.standard_normal(1000)
    p = torch.tensor(p0, requires_grad=True)
    opt = torch.optim.Adam([p], lr=3e-4, weight_decay=1e-4)
    q, m, v = p0.copy(), np.zeros_like(p0), np.zeros_like(p0)
    for step in range(1, 4):
        gr = g.standard_normal(1000) * 10.0 ** g.uniform(-9, 0, 1000)
        p.grad = torch.tensor(gr)
        opt.step()
        q, m, v = op.adam_step(q, gr, m, v, step, lr=3e-4, weight_decay=1e-4)
        assert np.abs(q - p.detach().numpy()).max() < 1e-12


def test_eval_forward_matches_reference():
    d = load("cnn_small_eval")
    sd = {k[6:]: d[k] for k in d.files if k.startswith("state/")}
    for B in (1, 4):
        e, _ = nm.forward(sd, d[f"b{B}/x"], train=False)
        assert np.abs(e - d[f"b{B}/emb"]).max() < 1e-5
        assert np.allclose(np.linalg.norm(e, axis=1), 1.0, atol=1e-6)


@pytest.mark.parametrize("name", MODEL_CASES)
def test_torch_port_matches_reference(name):
    """The fp32 torch-CPU port (timed CPU baseline) reproduces the reference's fp32 step."""
    import torch
    from oracle import torch_port as tp
    c = model_case(name)
    sd = {k: torch.tensor(v) for k, v in c["state0"].items()}
    for k in tp.param_names(sd):
        sd[k].requires_grad_(True)
    masks = [torch.tensor(m) for m in c["steps"][0]["masks"]]
    e = tp.forward(sd, torch.tensor(c["x"]), True, masks)
    loss = tp.supcon(e, torch.tensor(c["labels"]), c["temperature"], 0.07)
    loss.backward()
    assert np.abs(e.detach().numpy() - c["steps"][0]["emb"]).max() < 2e-6
    assert abs(loss.item() - c["steps"][0]["loss"]) < 2e-5
    got = {k: sd[k].grad.numpy() for k in tp.param_names(sd)}
    errs = grad_errors(got, c["grads"])
    errs64 = grad_errors(got, c["f64"]["grads"])
    for k in errs:
        assert min(errs[k][1], errs64[k][1]) < (2e-3 if errs[k][0] == "rel" else 1e-4), (k, errs[k])
