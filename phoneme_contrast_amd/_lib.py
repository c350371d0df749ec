"""ctypes binding of libpcx.so (the C ABI declared in include/pcx.h).

This is the one place Python touches the native library.  Nothing here falls back to a CPU or
PyTorch implementation: a missing library, a CPU tensor or a failing kernel raises.
"""
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# PCX_LIB_PATH: an alternative build of the same library (same-box A/B timing of kernel variants,
# scripts/ab_bench.sh); unset, the in-tree library
LIB_PATH = os.environ.get("PCX_LIB_PATH") or os.path.join(_HERE, "libpcx.so")

PCX_OK = 0
PCX_EINVAL = -1
PCX_ESHAPE = -2
PCX_EHIP = -3
PCX_EWORKSPACE = -5

REDUCTIONS = {"mean": 0, "sum": 1, "none": 2}

_lock = threading.Lock()
_lib = None

c_void_p = ctypes.c_void_p
c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_float = ctypes.c_float
c_size = ctypes.c_size_t



class NetConfig(ctypes.Structure):
    """pcx_net_config (include/pcx.h)."""
    _fields_ = [("kind", ctypes.c_int), ("in_channels", ctypes.c_int),
                ("embedding_dim", ctypes.c_int), ("use_attention", ctypes.c_int),
                ("hidden_dims", ctypes.c_int * 4), ("use_residual", ctypes.c_int),
                ("conv_bf16", ctypes.c_int)]


_pp = ctypes.POINTER(ctypes.c_void_p)
_pi = ctypes.POINTER(ctypes.c_int)
_ps = ctypes.POINTER(ctypes.c_size_t)

# name -> (restype, argtypes); mirrors include/pcx.h
SIGNATURES = {
    "pcx_version": (c_int, []),
    "pcx_last_error": (c_int, [ctypes.c_char_p, c_size]),
    "pcx_supcon_workspace_bytes": (c_size, [c_i64, c_i64]),
    "pcx_supcon_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_i64, c_i64, c_float, c_float,
                                   c_int, c_void_p, c_void_p, c_void_p, c_size, c_void_p]),
    "pcx_supcon_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_i64, c_i64, c_float, c_float,
                                    c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_size, c_void_p]),
    "pcx_supcon_rows_workspace_bytes": (c_size, [c_i64, c_i64, c_i64]),
    "pcx_supcon_forward_rows": (c_int, [c_void_p, c_void_p, c_void_p, c_i64, c_i64, c_i64, c_i64, c_float,
                                        c_float, c_int, c_void_p, c_void_p, c_void_p, c_size, c_void_p]),
    "pcx_supcon_coef_rows": (c_int, [c_void_p, c_void_p, c_i64, c_i64, c_float, c_int, c_void_p, c_void_p]),
    "pcx_supcon_backward_rows": (c_int, [c_void_p, c_void_p, c_void_p, c_i64, c_i64, c_i64, c_i64, c_float,
                                         c_float, c_void_p, c_void_p, c_void_p, c_size, c_void_p]),
    "pcx_adam_step": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_i64, c_float,
                              c_float, c_float, c_float, c_float, c_float, c_void_p]),
    "pcx_net_create": (c_void_p, [ctypes.POINTER(NetConfig), c_i64, c_i64, c_i64]),
    "pcx_net_destroy": (None, [c_void_p]),
    "pcx_net_workspace_bytes": (c_size, [c_void_p]),
    "pcx_net_info": (c_int, [c_void_p, _pi, _pi, _pi, _pi]),
    "pcx_net_region": (c_int, [c_void_p, ctypes.c_char_p, _ps, _ps]),
    "pcx_net_forward": (c_int, [c_void_p, _pp, _pp, _pp, c_void_p, _pp, c_int, c_void_p, c_void_p,
                                c_size, c_void_p]),
    "pcx_net_backward": (c_int, [c_void_p, _pp, c_void_p, _pp, c_void_p, c_void_p, _pp, c_void_p,
                                 c_size, c_void_p]),
    "pcx_net_profile": (c_int, [c_void_p, c_int]),
    "pcx_net_profile_only": (c_int, [c_void_p, ctypes.c_char_p]),
    "pcx_net_grad_buckets": (c_int, [c_void_p, c_int, _pi]),
    "pcx_net_bucket_wait": (c_int, [c_void_p, c_int, c_void_p]),
    "pcx_net_grad_stages": (c_int, [c_void_p, _pi, c_int]),
    "pcx_net_profile_read": (c_int, [c_void_p, ctypes.c_char_p, c_size, ctypes.POINTER(c_float), _pi,
                                     c_int]),
    "pcx_dropout_masks": (c_int, [c_void_p, c_i64, c_float, ctypes.c_uint64, ctypes.c_uint64,
                                  c_void_p]),
    "pcx_stream_copy": (c_int, [c_void_p, c_void_p, c_size, c_void_p]),
    "pcx_melspec": (c_int, [c_void_p, c_i64, c_i64, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                            c_int, c_void_p, c_void_p, c_void_p]),
    "pcx_mel_finish": (c_int, [c_void_p, c_void_p, c_i64, c_i64, c_int, c_int, c_float, c_void_p,
                               c_int, c_void_p, c_void_p, c_i64, c_void_p]),
    "pcx_compute_deltas": (c_int, [c_void_p, c_i64, c_void_p, c_i64, c_i64, c_int, c_i64,
                                   c_void_p]),
    "pcx_specaug": (c_int, [c_void_p, c_i64, c_int, c_i64, c_void_p, c_void_p, c_void_p, c_void_p,
                            ctypes.c_uint64, c_void_p]),
    "pcx_conv2d_workspace_bytes": (c_size, [c_int] * 8),
    "pcx_conv2d": (c_int, [c_int] * 12 + [c_void_p] * 4 + [c_int, c_void_p, c_size, c_void_p]),
}


class AugConfig(ctypes.Structure):
    """pcx_aug_config (include/pcx.h)."""
    _fields_ = [("time_enabled", c_int), ("time_width", c_int), ("time_prob", ctypes.c_double),
                ("freq_enabled", c_int), ("freq_width", c_int), ("freq_prob", ctypes.c_double),
                ("noise_enabled", c_int), ("noise_min", ctypes.c_double), ("noise_max", ctypes.c_double),
                ("noise_prob", ctypes.c_double)]


SIGNATURES["pcx_draw_view_params"] = (c_int, [c_void_p, c_void_p, c_i64, c_int, c_int,
                                              ctypes.POINTER(AugConfig), c_void_p, c_void_p,
                                              c_void_p, c_void_p])


class PcxError(RuntimeError):
    """A libpcx call failed (HIP error, bad workspace, ...)."""


def lib():
    """Load libpcx.so once; raise if it is missing (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"phoneme_contrast_amd: native library {LIB_PATH} is missing; build it with "
                    "`make` (or __graft_entry__.build()) — there is no CPU fallback")
            handle = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
    return _lib


def last_error():
    buf = ctypes.create_string_buffer(512)
    lib().pcx_last_error(buf, 512)
    return buf.value.decode(errors="replace")


def check(rc, what):
    if rc == PCX_OK:
        return
    msg = last_error()
    if rc == PCX_EINVAL or rc == PCX_ESHAPE:
        raise ValueError(msg or what)
    raise PcxError(f"{what} failed ({rc}): {msg}")


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def stream_of(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def require_gpu(*tensors, what="phoneme_contrast_amd"):
    for t in tensors:
        if t is not None and t.device.type != "cuda":
            raise RuntimeError(
                f"{what}: tensors must live on a ROCm GPU (got device '{t.device}'); the "
                "MI355X kernels have no CPU path")


def workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
