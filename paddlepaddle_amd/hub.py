"""paddle.hub (reference python/paddle/hub.py): list / help / load entry points of a ``hubconf.py``.
Only ``source='local'`` works here (no network for github / gitee)."""
from __future__ import annotations

import importlib.util
import os
import sys

__all__ = ["list", "help", "load"]

_builtin_list = list


def _load_hubconf(repo_dir, source):
    if source != "local":
        raise RuntimeError(f"paddle.hub source={source!r} needs network access; use source='local'")
    path = os.path.join(repo_dir, "hubconf.py")
    if not os.path.exists(path):
        raise FileNotFoundError(f"no hubconf.py in {repo_dir}")
    spec = importlib.util.spec_from_file_location("hubconf", path)
    mod = importlib.util.module_from_spec(spec)
    sys.path.insert(0, repo_dir)
    try:
        spec.loader.exec_module(mod)
    finally:
        sys.path.remove(repo_dir)
    return mod


def list(repo_dir, source="github", force_reload=False):  # noqa: A001
    mod = _load_hubconf(repo_dir, source)
    return [n for n in dir(mod) if callable(getattr(mod, n)) and not n.startswith("_")]


def help(repo_dir, model, source="github", force_reload=False):  # noqa: A001
    return getattr(_load_hubconf(repo_dir, source), model).__doc__


def load(repo_dir, model, source="github", force_reload=False, **kwargs):
    return getattr(_load_hubconf(repo_dir, source), model)(**kwargs)
