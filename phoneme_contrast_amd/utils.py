"""Device / logging / resource helpers with the reference's names and semantics
(src/utils/device.py:9-64, logging.py:6-47, system_resources.py:37-82)."""
import logging
import multiprocessing
import os
from pathlib import Path
from typing import Optional

import torch


def get_best_device(device_str: str = "auto", logger: Optional[logging.Logger] = None) -> torch.device:
    """'auto' -> cuda:0 (a ROCm GPU; 'cuda' is HIP under PyTorch-ROCm) when present, else CPU with
    cores-2 threads as the reference does.  The MI355X kernels need the GPU; a CPU device makes
    the model raise on its first forward."""
    log = logger.info if logger else print
    if device_str != "auto":
        log(f"Using explicitly requested device: {device_str}")
        return torch.device(device_str)
    if torch.cuda.is_available():
        n = torch.cuda.device_count()
        log(f"Found {n} ROCm GPU device(s)")
        # N ranks rehearsed on fewer GPUs (PCX_DIST_BACKEND=gloo) share them round-robin
        from .distributed import local_device_index
        local = local_device_index(int(os.environ.get("LOCAL_RANK", "0")), n)
        props = torch.cuda.get_device_properties(local)
        log(f"Selected GPU {local}: {props.name}")
        return torch.device(f"cuda:{local}")
    log("No GPU found, using CPU")
    cpu = os.cpu_count()
    if cpu:
        torch.set_num_threads(max(1, cpu - 2))
    return torch.device("cpu")


def create_logger(log_dir: Path, console_log_level: str = "info") -> logging.Logger:
    """logs/log_info.txt (INFO+), logs/log_debug.txt (DEBUG+) and the console."""
    log_dir = Path(log_dir)
    log_dir.mkdir(parents=True, exist_ok=True)
    logger = logging.getLogger("experiment_logger")
    logger.setLevel(logging.DEBUG)
    logger.handlers.clear()
    logger.propagate = False
    fmt = logging.Formatter("[%(asctime)s] [%(levelname)s] %(message)s", "%Y-%m-%d %H:%M:%S")
    for path, level in ((log_dir / "log_info.txt", logging.INFO), (log_dir / "log_debug.txt", logging.DEBUG)):
        h = logging.FileHandler(path)
        h.setLevel(level)
        h.setFormatter(fmt)
        logger.addHandler(h)
    c = logging.StreamHandler()
    c.setLevel(logging.DEBUG if console_log_level == "debug" else logging.INFO)
    c.setFormatter(fmt)
    logger.addHandler(c)
    return logger


def get_logger() -> logging.Logger:
    return logging.getLogger("experiment_logger")


def adjust_params_for_system(cfg, device: torch.device, logger: Optional[logging.Logger] = None):
    """num_workers = min(4, cores-1) when 0, pin_memory = (device is GPU) when null."""
    import copy
    cfg = copy.deepcopy(cfg)
    cores = multiprocessing.cpu_count()
    if cfg.training.num_workers == 0:
        cfg.training.num_workers = min(4, cores - 1)
    if cfg.training.pin_memory is None:
        cfg.training.pin_memory = device.type == "cuda"
    if logger:
        logger.debug(f"CPU cores: {cores}, num_workers: {cfg.training.num_workers}, "
                     f"pin_memory: {cfg.training.pin_memory}")
    return cfg
