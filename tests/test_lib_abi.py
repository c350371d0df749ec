"""CPU-side checks of the C ABI: libpcx.so loads and exports every symbol include/pcx.h declares,
and the ctypes table mirrors the header.  No kernel is launched here."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pcx.h")
LIB = os.path.join(ROOT, "phoneme_contrast_amd", "libpcx.so")


def declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pcx_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def so():
    if not os.path.exists(LIB):
        pytest.fail("libpcx.so not built (run `make` or __graft_entry__.build())")
    return ctypes.CDLL(LIB)


def test_header_declares_api():
    names = declared()
    assert "pcx_supcon_forward" in names and "pcx_adam_step" in names


def test_library_exports_every_declared_symbol(so):
    missing = [n for n in declared() if not hasattr(so, n)]
    assert not missing, missing


def test_ctypes_table_matches_header():
    from phoneme_contrast_amd import _lib
    assert sorted(_lib.SIGNATURES) == declared()


def test_version_and_error_channel(so):
    so.pcx_version.restype = ctypes.c_int
    assert so.pcx_version() >= 100
    so.pcx_supcon_workspace_bytes.restype = ctypes.c_size_t
    so.pcx_supcon_workspace_bytes.argtypes = [ctypes.c_int64, ctypes.c_int64]
    assert so.pcx_supcon_workspace_bytes(4096, 128) > 0


def test_invalid_arguments_rejected_without_gpu(so):
    """Argument validation runs before any HIP call, so it is testable on CPU."""
    from phoneme_contrast_amd import _lib
    lib = _lib.lib()
    rc = lib.pcx_supcon_forward(None, None, None, 8, 128, 0.1, 0.07, 0, None, None, None, 0, None)
    assert rc == _lib.PCX_EINVAL
    assert "features is NULL" in _lib.last_error()
    rc = lib.pcx_adam_step(None, None, None, None, 10, 1, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1.0, None)
    assert rc == _lib.PCX_EINVAL


def test_cpu_tensor_fails_loudly():
    import torch
    from phoneme_contrast_amd.losses import SupervisedContrastiveLoss
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        SupervisedContrastiveLoss()(torch.randn(4, 128), torch.tensor([0, 0, 1, 1]))
