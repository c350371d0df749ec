"""One rank of `scripts/train.py main()` launched by torch.distributed.run (tests/test_entry_dist_gpu.py).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
        tests/dist_train_worker.py OUT_DIR override [override ...]

Composes the configs/ tree with the overrides (experiment.output_dir = OUT_DIR/run), runs the entry's
main() exactly as `python scripts/train.py` would under torchrun, then writes this rank's final
parameters, buffers and loss history to OUT_DIR/rank<r>.npz.
"""
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    out_dir, overrides = sys.argv[1], sys.argv[2:]
    from phoneme_contrast_amd import config as cfglib
    cfg = cfglib.compose(os.path.join(ROOT, "configs"), "config", overrides,
                         output_dir=os.path.join(out_dir, "run"))
    spec = importlib.util.spec_from_file_location("pcx_train_entry", os.path.join(ROOT, "scripts", "train.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    tr = mod.main(cfg)
    rank = int(os.environ.get("RANK", "0"))
    out = {f"p/{k}": v.detach().cpu().numpy() for k, v in tr.model.state_dict().items()}
    out["train_loss"] = np.asarray(tr.metrics_history["train_loss"], np.float64)
    out["global_step"] = np.array([tr.global_step])
    out["bucketer"] = np.array([getattr(tr.model, "_grad_bucketer", None) is not None])
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **out)
    print(f"rank {rank}: ok", flush=True)


if __name__ == "__main__":
    main()
