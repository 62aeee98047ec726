"""Native ops: loader for the in-tree extension ``ddlb_amd._C``.

``load()`` imports torch FIRST (so the extension's ``libamdhip64.so.7`` / ``librccl.so.1`` resolve
to the copies torch ships), then the extension. On a GPU box a missing or stale extension is an
error, never a silent PyTorch fallback.
"""

from __future__ import annotations

import importlib
import os

_C = None


class NativeUnavailable(RuntimeError):
    pass


def load(build_if_missing: bool = None):
    """Return the ``_C`` module, building it in-tree first if allowed and needed."""
    global _C
    if _C is not None:
        return _C
    import torch  # noqa: F401  (must precede the extension, see module docstring)

    if build_if_missing is None:
        build_if_missing = os.environ.get("DDLB_AUTOBUILD", "1") == "1"
    try:
        _C = importlib.import_module("ddlb_amd._C")
    except ImportError as first:
        if not build_if_missing:
            raise NativeUnavailable(
                "ddlb_amd._C is not built; run `python -m ddlb_amd._build`") from first
        from ddlb_amd import _build

        _build.build()
        importlib.invalidate_caches()
        _C = importlib.import_module("ddlb_amd._C")
    return _C


def available() -> bool:
    try:
        load(build_if_missing=False)
        return True
    except Exception:
        return False
