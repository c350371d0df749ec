"""Hydra-compatible config composition for the `configs/` tree (no hydra/omegaconf needed).

The reference drives everything through `@hydra.main(config_path="../configs",
config_name="config")` (scripts/train.py:150-151).  hydra-core / omegaconf are not installed in
this image, so `compose()` implements the subset the reference's configs use:

  * defaults list with `_self_` and config groups (`data: default`, `model: cnn_small`, ...);
    `_self_` first means the primary file is applied first and group files override it;
  * command-line overrides `key.path=value`, `group=option`, `+new.key=value`, `~key`;
  * `${a.b}` interpolation and `${hydra:runtime.output_dir}` (outputs/<date>/<time>);
  * an attribute-access config object with `.get`, `dict(...)`, `to_container()`, `to_yaml()`.
When hydra *is* importable, scripts/train.py composes with @hydra.main instead and wraps the
resolved container with `wrap()`.
"""
import copy
import datetime
import os
import re

import yaml


class Cfg(dict):
    """dict with attribute access (DictConfig stand-in)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def __deepcopy__(self, memo):
        return Cfg({k: copy.deepcopy(v, memo) for k, v in self.items()})


def _wrap(x):
    if isinstance(x, dict):
        return Cfg({k: _wrap(v) for k, v in x.items()})
    if isinstance(x, list):
        return [_wrap(v) for v in x]
    return x


def wrap(d):
    """Attribute-access config from a plain (resolved) container, e.g. OmegaConf.to_container."""
    return _wrap(d)


def to_container(cfg):
    if isinstance(cfg, dict):
        return {k: to_container(v) for k, v in cfg.items()}
    if isinstance(cfg, list):
        return [to_container(v) for v in cfg]
    return cfg


def to_yaml(cfg):
    return yaml.safe_dump(to_container(cfg), sort_keys=False)


def _merge(dst, src):
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


class _Loader(yaml.SafeLoader):
    """YAML 1.1 safe loader that, like OmegaConf's, also reads `3e-4` / `1e-6` as floats."""


_Loader.add_implicit_resolver(
    "tag:yaml.org,2002:float",
    re.compile(r"""^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
                  |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
                  |\.[0-9_]+(?:[eE][-+][0-9]+)?
                  |[-+]?\.(?:inf|Inf|INF)
                  |\.(?:nan|NaN|NAN))$""", re.X),
    list("-+0123456789."))


def _load(path):
    with open(path) as f:
        return yaml.load(f, Loader=_Loader) or {}


def _parse_value(s):
    try:
        return yaml.load(s, Loader=_Loader)
    except yaml.YAMLError:
        return s


def _set(cfg, dotted, value, create):
    keys = dotted.split(".")
    node = cfg
    for k in keys[:-1]:
        if k not in node:
            if not create:
                raise KeyError(f"Could not override '{dotted}': key '{k}' not in config (use +{dotted}=...)")
            node[k] = {}
        node = node[k]
    if keys[-1] not in node and not create:
        raise KeyError(f"Could not override '{dotted}': key not in config (use +{dotted}=...)")
    node[keys[-1]] = value


def _get(cfg, dotted):
    node = cfg
    for k in dotted.split("."):
        node = node[k]
    return node


_INTERP = re.compile(r"\$\{([^}]+)\}")


def _resolve(cfg, root, runtime):
    if isinstance(cfg, dict):
        for k in list(cfg):
            cfg[k] = _resolve(cfg[k], root, runtime)
        return cfg
    if isinstance(cfg, list):
        return [_resolve(v, root, runtime) for v in cfg]
    if isinstance(cfg, str) and "${" in cfg:
        def sub(m):
            key = m.group(1)
            if key.startswith("hydra:"):
                return str(runtime.get(key[6:], ""))
            return str(_get(root, key))
        full = _INTERP.fullmatch(cfg)
        if full and not full.group(1).startswith("hydra:"):
            return _get(root, full.group(1))
        return _INTERP.sub(sub, cfg)
    return cfg


def compose(config_dir, config_name="config", overrides=(), output_dir=None):
    """Compose `config_dir/config_name.yaml` with its defaults list and CLI overrides."""
    primary = _load(os.path.join(config_dir, config_name + ".yaml"))
    defaults = primary.pop("defaults", ["_self_"])
    groups = {}
    order = []
    for d in defaults:
        if d == "_self_":
            order.append(("_self_", None))
        elif isinstance(d, dict):
            (g, opt), = d.items()
            groups[g] = opt
            order.append((g, opt))
    plain = []
    for ov in overrides:
        k, _, v = ov.partition("=")
        if not k.startswith(("+", "~")) and "." not in k and k in groups:
            groups[k] = v
        else:
            plain.append(ov)
    cfg = {}
    for g, _ in order:
        if g == "_self_":
            _merge(cfg, primary)
        else:
            opt = groups[g]
            path = os.path.join(config_dir, g, f"{opt}.yaml")
            if not os.path.exists(path):
                avail = sorted(f[:-5] for f in os.listdir(os.path.join(config_dir, g)) if f.endswith(".yaml"))
                raise ValueError(f"Could not find '{g}/{opt}'. Available options in '{g}': {avail}")
            _merge(cfg.setdefault(g, {}), _load(path))
    for ov in plain:
        k, _, v = ov.partition("=")
        if k.startswith("~"):
            keys = k[1:].split(".")
            node = cfg
            for kk in keys[:-1]:
                node = node[kk]
            node.pop(keys[-1], None)
        elif k.startswith("+"):
            _set(cfg, k.lstrip("+"), _parse_value(v), create=True)
        else:
            _set(cfg, k, _parse_value(v), create=False)
    if output_dir is None:
        now = datetime.datetime.now()
        output_dir = os.path.join("outputs", now.strftime("%Y-%m-%d"), now.strftime("%H-%M-%S"))
    _resolve(cfg, cfg, {"runtime.output_dir": output_dir})
    return _wrap(cfg)
