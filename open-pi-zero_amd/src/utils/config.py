"""Config access without omegaconf/hydra (neither is installed on the MI355X image).

``cfg_get(cfg, "a.b", default)`` works on OmegaConf nodes, plain dicts and
attribute objects alike.  ``load_config(path, overrides)`` reads a
bridge.yaml-style file (config/train/bridge.yaml in the reference) with PyYAML
and resolves the interpolations the hot-path keys use: ``${a.b}``,
``${eval:'expr'}``, ``${oc.env:VAR}`` (empty if unset) and ``${now:...}``.
``instantiate(node, **kw)`` resolves ``_target_`` like hydra.utils.instantiate.
"""

from __future__ import annotations

import importlib
import os
import re
import time

import yaml


class AttrDict(dict):
    """dict with attribute access, recursive, OmegaConf-DictConfig-like ``.get``."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    @staticmethod
    def wrap(x):
        if isinstance(x, dict) and not isinstance(x, AttrDict):
            return AttrDict({k: AttrDict.wrap(v) for k, v in x.items()})
        if isinstance(x, list):
            return [AttrDict.wrap(v) for v in x]
        return x


def cfg_get(cfg, key, default=None):
    cur = cfg
    for part in key.split("."):
        if cur is None:
            return default
        if isinstance(cur, dict):
            if part not in cur:
                return default
            cur = cur[part]
        else:
            try:
                cur = getattr(cur, part)
            except AttributeError:
                try:
                    cur = cur.get(part, None)
                except Exception:
                    return default
                if cur is None:
                    return default
    return default if cur is None else cur


_REF = re.compile(r"\$\{([^${}]+)\}")


def _lookup(root, path):
    cur = root
    for p in path.split("."):
        cur = cur[p]
    return cur


def _resolve_str(s, root, depth=0):
    if depth > 20 or not isinstance(s, str) or "${" not in s:
        return s

    def rep(m):
        expr = m.group(1).strip()
        if expr.startswith("oc.env:"):
            return os.environ.get(expr[len("oc.env:"):].split(",")[0].strip(), "")
        if expr.startswith("now:"):
            return time.strftime(expr[len("now:"):])
        if expr.startswith("eval:"):
            inner = _resolve_str(expr[len("eval:"):].strip().strip("'\""), root, depth + 1)
            return str(eval(inner, {"__builtins__": {}}, {}))  # noqa: S307 (trusted config)
        v = _resolve_str(_lookup(root, expr), root, depth + 1)
        return v if isinstance(v, str) else repr(v) if not isinstance(v, (int, float)) else str(v)

    whole = _REF.fullmatch(s.strip())
    if whole and not whole.group(1).startswith(("oc.env:", "now:", "eval:")):
        v = _lookup(root, whole.group(1).strip())
        if isinstance(v, (dict, list)):
            return _resolve(v, root)
        return _resolve_str(v, root, depth + 1) if isinstance(v, str) else v
    out = _REF.sub(rep, s)
    return _resolve_str(out, root, depth + 1) if "${" in out else _coerce(out)


def _coerce(v):
    if isinstance(v, str):
        try:
            if re.fullmatch(r"[-+]?\d+", v):
                return int(v)
            return float(v) if re.fullmatch(r"[-+]?(\d+\.?\d*|\.\d+)([eE][-+]?\d+)?", v) else v
        except ValueError:
            return v
    return v


def _resolve(node, root):
    if isinstance(node, dict):
        return {k: _resolve(v, root) for k, v in node.items()}
    if isinstance(node, list):
        return [_resolve(v, root) for v in node]
    return _coerce(_resolve_str(node, root))


def load_config(path, overrides=None):
    with open(path) as f:
        raw = yaml.safe_load(f)
    for k, v in (overrides or {}).items():
        cur = raw
        parts = k.split(".")
        for p in parts[:-1]:
            cur = cur.setdefault(p, {})
        cur[parts[-1]] = v
    return AttrDict.wrap(_resolve(raw, raw))


def instantiate(node, **kw):
    mod, cls = cfg_get(node, "_target_").rsplit(".", 1)
    args = {k: v for k, v in dict(node).items() if k != "_target_"}
    args.update(kw)
    return getattr(importlib.import_module(mod), cls)(**args)
