"""Model plugin registry and the phoneme CNNs — drop-in for reference src/models/.

`model_registry`, `BaseModel`, `PhonemeNet` ("phoneme_cnn") and `PhonemeNetDeep`
("phoneme_cnn_deep") keep the reference's names, config keys, defaults, initialisation and
state_dict keys/shapes (so checkpoints interoperate, reference src/models/phoneme_cnn.py and
scripts/evaluate.py:271-277).  The nn.Conv2d / nn.BatchNorm2d / nn.Linear children are parameter
*holders* only: forward and backward run as one libpcx call each (csrc/net.hip), with every
conv, BN, ReLU, MaxPool, Dropout2d, attention, pooling, projection and normalize fused into
hand-written gfx950 kernels.  There is no CPU path: a CPU tensor raises.
"""
import ctypes
from typing import Callable, Dict, List, Optional, Type

import torch
import torch.nn as nn

from . import _lib


# ----------------------------------------------------------------------------- registry
class ModelRegistry:
    """name -> model class (reference src/models/registry.py:7-41)."""

    def __init__(self):
        self._models: Dict[str, Type["BaseModel"]] = {}

    def register(self, name: str) -> Callable:
        def decorator(cls):
            if name in self._models:
                raise ValueError(f"Model {name} already registered")
            self._models[name] = cls
            return cls
        return decorator

    def get(self, name: str) -> Type["BaseModel"]:
        if name not in self._models:
            raise ValueError(f"Model {name} not found. Available: {list(self._models.keys())}")
        return self._models[name]

    def create(self, name: str, config: Dict) -> "BaseModel":
        return self.get(name)(config)

    def list(self) -> List[str]:
        return list(self._models.keys())


model_registry = ModelRegistry()


class BaseModel(nn.Module):
    """Base class keeping `self.config` (reference src/models/base.py:9-31)."""

    def __init__(self, config: Dict):
        super().__init__()
        self.config = config

    def forward(self, x: torch.Tensor) -> torch.Tensor:  # pragma: no cover - abstract
        raise NotImplementedError

    def get_embedding_dim(self) -> int:
        return self.config.get("embedding_dim", 128)


# ----------------------------------------------------------------------------- native runner
def _ptr_array(tensors, ctype=ctypes.c_void_p):
    arr = (ctype * len(tensors))()
    for i, t in enumerate(tensors):
        arr[i] = t.data_ptr() if t is not None else None
    return arr


class _Plan:
    """Owns one pcx_net plan (host object) for a fixed (config, B, F, T)."""

    def __init__(self, cfg: "_lib.NetConfig", B: int, F: int, T: int):
        lib = _lib.lib()
        self.handle = lib.pcx_net_create(ctypes.byref(cfg), B, F, T)
        if not self.handle:
            raise ValueError(_lib.last_error())
        self.ws_bytes = lib.pcx_net_workspace_bytes(self.handle)
        np_, nbn, ndrop = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        ch = (ctypes.c_int * 8)()
        _lib.check(lib.pcx_net_info(self.handle, ctypes.byref(np_), ctypes.byref(nbn),
                                    ctypes.byref(ndrop), ch), "pcx_net_info")
        self.nparams, self.nbn, self.ndrop = np_.value, nbn.value, ndrop.value
        self.drop_channels = [ch[i] for i in range(self.ndrop)]

    def region(self, ws: torch.Tensor, name: str, shape) -> torch.Tensor:
        off, nb = ctypes.c_size_t(), ctypes.c_size_t()
        _lib.check(_lib.lib().pcx_net_region(self.handle, name.encode(), ctypes.byref(off),
                                             ctypes.byref(nb)), "pcx_net_region")
        return ws[off.value:off.value + nb.value].view(torch.float32).view(*shape)

    def __del__(self):
        try:
            if self.handle:
                _lib.lib().pcx_net_destroy(self.handle)
        except Exception:
            pass


class _NetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, x, *params):
        emb, ws, plan, masks = model._native_forward(x, params)
        ctx.model, ctx.ws, ctx.plan, ctx.masks = model, ws, plan, masks
        ctx.save_for_backward(x, emb, *params)
        return emb

    @staticmethod
    def backward(ctx, demb):
        x, emb, *params = ctx.saved_tensors
        grads = ctx.model._native_backward(ctx.plan, ctx.ws, x, emb, demb, params, ctx.masks)
        ctx.ws = None
        return (None, None, *grads)


class _NativeNet(BaseModel):
    """Shared host logic of PhonemeNet / PhonemeNetDeep: plan cache, pointer marshalling,
    dropout masks, autograd glue."""

    _kind = None

    def __init__(self, config):
        super().__init__(config)
        self._plans = {}
        self._next_masks = None
        self.last_dropout_masks = None
        self._grad_bucketer = None

    # --- configuration handed to the native plan
    def _net_config(self) -> "_lib.NetConfig":
        raise NotImplementedError

    def _bn_modules(self):
        return [m for m in self.modules() if isinstance(m, (nn.BatchNorm2d, nn.BatchNorm1d))]

    def _plan(self, B, F, T):
        key = (B, F, T)
        p = self._plans.get(key)
        if p is None:
            p = _Plan(self._net_config(), B, F, T)
            if getattr(self, "_profiling", False):
                _lib.check(_lib.lib().pcx_net_profile(p.handle, 1), "pcx_net_profile")
                only = getattr(self, "_profile_only", None)
                _lib.check(_lib.lib().pcx_net_profile_only(p.handle, only.encode() if only else None),
                           "pcx_net_profile_only")
            if p.nparams != len(list(self.parameters())):
                raise RuntimeError("native plan / module parameter count mismatch")
            self._plans[key] = p
        return p

    def kernel_profile(self, enable: bool = True, only: Optional[str] = None):
        """Start (or stop) per-launch HIP-event timing of the native kernels (all cached plans);
        only: record that kernel label alone (one event pair per launch of it)."""
        lib = _lib.lib()
        self._profiling = bool(enable)
        self._profile_only = only
        for p in self._plans.values():
            _lib.check(lib.pcx_net_profile(p.handle, 1 if enable else 0), "pcx_net_profile")
            _lib.check(lib.pcx_net_profile_only(p.handle, only.encode() if only else None), "pcx_net_profile_only")

    def kernel_profile_read(self):
        """{kernel label: (total_ms, launches)} since kernel_profile(True); waits for the events."""
        lib = _lib.lib()
        out = {}
        for p in self._plans.values():
            buf = ctypes.create_string_buffer(8192)
            ms = (ctypes.c_float * 256)()
            cnt = (ctypes.c_int * 256)()
            n = lib.pcx_net_profile_read(p.handle, buf, 8192, ms, cnt, 256)
            if n < 0:
                _lib.check(n, "pcx_net_profile_read")
            for i, lab in enumerate(buf.value.decode().split("\n")[:n]):
                t, c = out.get(lab, (0.0, 0))
                out[lab] = (t + ms[i], c + cnt[i])
        return out

    def set_dropout_masks(self, masks: Optional[List[torch.Tensor]]):
        """Inject the Dropout2d keep-scale masks ([B, C] each, 0 or 1/(1-p)) used by the next
        training forward (parity tests replay the reference's masks this way)."""
        self._next_masks = masks

    def _dropout_masks(self, plan, B, device):
        if not self.training:
            return None
        if self._next_masks is not None:
            masks = [m.to(device=device, dtype=torch.float32).contiguous() for m in self._next_masks]
            self._next_masks = None
            return masks
        p = float(self.dropout_rate)
        if p <= 0.0:
            return None
        if p >= 1.0:
            return [torch.zeros(B, c, device=device) for c in plan.drop_channels]
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        masks = []
        lib = _lib.lib()
        stream = _lib.stream_of(torch.empty(0, device=device))
        for i, c in enumerate(plan.drop_channels):
            m = torch.empty(B, c, device=device)
            _lib.check(lib.pcx_dropout_masks(_lib.ptr(m), B * c, p, seed, i << 40, stream),
                       "pcx_dropout_masks")
            masks.append(m)
        return masks

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        _lib.require_gpu(x, what=type(self).__name__)
        if x.dim() != 4 or x.shape[1] != self.in_channels:
            raise ValueError(f"expected input [batch, {self.in_channels}, n_mfcc, time], got {tuple(x.shape)}")
        for p in self.parameters():
            if p.device != x.device or p.dtype != torch.float32:
                raise RuntimeError(f"{type(self).__name__}: parameters must be float32 on {x.device}")
        if self.training and x.shape[0] == 1:
            raise ValueError("Expected more than 1 value per channel when training, got input size "
                             f"torch.Size([1, {self.embedding_dim}])")
        x = x.contiguous().float()
        params = tuple(self.parameters())
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return _NetFn.apply(self, x, *params)
        emb, _, _, _ = self._native_forward(x, params)
        return emb

    def _native_forward(self, x, params):
        B, _, F, T = x.shape
        plan = self._plan(B, F, T)
        lib = _lib.lib()
        ws = torch.empty(plan.ws_bytes, dtype=torch.uint8, device=x.device)
        emb = torch.empty(B, self.embedding_dim, device=x.device, dtype=torch.float32)
        bns = self._bn_modules()
        stats, counts = [], []
        for m in bns:
            stats += [m.running_mean, m.running_var]
            counts.append(m.num_batches_tracked)
        masks = self._dropout_masks(plan, B, x.device)
        self.last_dropout_masks = masks
        pa = _ptr_array([p.detach() for p in params])
        sa = _ptr_array(stats)
        ca = _ptr_array(counts)
        da = _ptr_array(masks) if masks is not None else None
        _lib.check(lib.pcx_net_forward(plan.handle, pa, sa, ca, _lib.ptr(x), da,
                                       1 if self.training else 0, _lib.ptr(emb), _lib.ptr(ws),
                                       plan.ws_bytes, _lib.stream_of(x)), "pcx_net_forward")
        return emb, ws, plan, masks

    def _native_backward(self, plan, ws, x, emb, demb, params, masks):
        lib = _lib.lib()
        sizes = [p.numel() for p in params]
        flat = torch.empty(sum(sizes), device=x.device, dtype=torch.float32)
        grads, off = [], 0
        for p, n in zip(params, sizes):
            grads.append(flat[off:off + n].view_as(p))
            off += n
        da = _ptr_array(masks) if masks is not None else None
        g_emb = demb.contiguous().float()  # held until the launch is enqueued
        bucketer = getattr(self, "_grad_bucketer", None)
        if bucketer is not None:
            bucketer.prepare(plan)
        _lib.check(lib.pcx_net_backward(plan.handle, _ptr_array([p.detach() for p in params]),
                                        _lib.ptr(x), da, _lib.ptr(emb),
                                        _lib.ptr(g_emb), _ptr_array(grads),
                                        _lib.ptr(ws), plan.ws_bytes, _lib.stream_of(x)),
                   "pcx_net_backward")
        if bucketer is not None:  # DDP: bucket all-reduces start behind the layers still running
            bucketer.launch(plan, flat)
        return grads

    # initialisation shared by both nets (reference phoneme_cnn.py:79-96, :259-272)
    def _initialize_weights(self) -> None:
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, (nn.BatchNorm2d, nn.BatchNorm1d)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0, 0.01)
                nn.init.constant_(m.bias, 0)


class SpatialAttention(nn.Module):
    """1x1 conv -> sigmoid gate (reference phoneme_cnn.py:129-143); parameter holder."""

    def __init__(self, in_channels: int):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, 1, kernel_size=1)


def _double_conv(cin, cout, p, pool):
    """conv-BN-ReLU x2 (+ MaxPool2d(2)) + Dropout2d, child indices as the reference's blocks."""
    layers = [nn.Conv2d(cin, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True),
              nn.Conv2d(cout, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True)]
    if pool:
        layers.append(nn.MaxPool2d(2, 2))
    layers.append(nn.Dropout2d(p))
    return nn.Sequential(*layers)


@model_registry.register("phoneme_cnn")
class PhonemeNet(_NativeNet):
    """cnn_small (reference src/models/phoneme_cnn.py:10-126): 3 conv blocks 1->32->64->128,
    SpatialAttention, global average pool, Linear+BatchNorm1d, L2 normalisation."""

    _kind = 0

    def __init__(self, config: dict):
        super().__init__(config)
        self.in_channels = config.get("in_channels", 1)
        self.embedding_dim = config.get("embedding_dim", 128)
        self.use_attention = config.get("use_attention", True)
        self.dropout_rate = config.get("dropout_rate", 0.1)
        self._build_network()
        self._initialize_weights()

    def _build_network(self) -> None:
        p = self.dropout_rate
        self.conv_blocks = nn.ModuleList([
            _double_conv(self.in_channels, 32, p, True),
            _double_conv(32, 64, p, True),
            _double_conv(64, 128, p, False),
        ])
        if self.use_attention:
            self.attention = SpatialAttention(128)
        self.global_pool = nn.AdaptiveAvgPool2d(1)
        self.projection = nn.Sequential(nn.Linear(128, self.embedding_dim),
                                        nn.BatchNorm1d(self.embedding_dim))

    def _net_config(self):
        cfg = _lib.NetConfig()
        cfg.kind = self._kind
        cfg.in_channels = self.in_channels
        cfg.embedding_dim = self.embedding_dim
        cfg.use_attention = 1 if self.use_attention else 0
        return cfg


class ResidualBlock(nn.Module):
    """Residual block parameter holder (reference phoneme_cnn.py:146-184): conv3x3(stride) + BN +
    ReLU, Dropout2d, conv3x3 + BN, shortcut = identity or conv1x1(stride) + BN, add, ReLU."""

    def __init__(self, in_channels, out_channels, stride=1, dropout_rate=0.1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, stride=stride, padding=1)
        self.bn1 = nn.BatchNorm2d(out_channels)
        self.conv2 = nn.Conv2d(out_channels, out_channels, 3, padding=1)
        self.bn2 = nn.BatchNorm2d(out_channels)
        self.dropout = nn.Dropout2d(dropout_rate)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_channels != out_channels:
            self.shortcut = nn.Sequential(nn.Conv2d(in_channels, out_channels, 1, stride=stride),
                                          nn.BatchNorm2d(out_channels))


@model_registry.register("phoneme_cnn_deep")
class PhonemeNetDeep(_NativeNet):
    """cnn_deep (reference src/models/phoneme_cnn.py:187-304): 7x7 stem + MaxPool(3,2,1), four
    ResidualBlocks (strides 1,2,2,2), SpatialAttention, pool, Linear+BatchNorm1d, normalize."""

    _kind = 1

    def __init__(self, config: dict):
        super().__init__(config)
        self.in_channels = config.get("in_channels", 1)
        self.embedding_dim = config.get("embedding_dim", 128)
        self.use_attention = config.get("use_attention", True)
        self.dropout_rate = config.get("dropout_rate", 0.2)
        self.hidden_dims = list(config.get("hidden_dims", [64, 128, 256, 512]))
        self.use_residual = config.get("use_residual", True)
        # MI355X addition: "bf16" runs every convolution on bf16 operands with float32 accumulation
        # (SURVEY 8(f) row 2); parameters, activations, statistics and gradients stay float32
        self.precision = config.get("precision", "fp32")
        if self.precision not in ("fp32", "bf16"):
            raise ValueError(f"PhonemeNetDeep: precision {self.precision!r} (fp32 | bf16)")
        self._build_network()
        self._initialize_weights()

    def _build_network(self) -> None:
        h = self.hidden_dims
        self.init_conv = nn.Sequential(nn.Conv2d(self.in_channels, h[0], 7, stride=1, padding=3),
                                       nn.BatchNorm2d(h[0]), nn.ReLU(inplace=True),
                                       nn.MaxPool2d(3, stride=2, padding=1))
        blocks, cin = [], h[0]
        for i, cout in enumerate(h):
            s = 1 if i == 0 else 2
            if self.use_residual:
                blocks.append(ResidualBlock(cin, cout, s, self.dropout_rate))
            else:  # reference phoneme_cnn.py:230-243
                blocks.append(nn.Sequential(
                    nn.Conv2d(cin, cout, 3, stride=s, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True),
                    nn.Conv2d(cout, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True),
                    nn.Dropout2d(self.dropout_rate)))
            cin = cout
        self.conv_blocks = nn.Sequential(*blocks)
        if self.use_attention:
            self.attention = SpatialAttention(h[-1])
        self.global_pool = nn.AdaptiveAvgPool2d(1)
        self.projection = nn.Sequential(nn.Linear(h[-1], self.embedding_dim),
                                        nn.BatchNorm1d(self.embedding_dim))

    def _net_config(self):
        cfg = _lib.NetConfig()
        cfg.kind = self._kind
        cfg.in_channels = self.in_channels
        cfg.embedding_dim = self.embedding_dim
        cfg.use_attention = 1 if self.use_attention else 0
        for i, d in enumerate(self.hidden_dims[:4]):
            cfg.hidden_dims[i] = d
        cfg.use_residual = 1 if self.use_residual else 0
        cfg.conv_bf16 = 1 if self.precision == "bf16" else 0
        return cfg
