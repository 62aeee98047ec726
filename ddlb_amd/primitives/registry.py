"""Implementation registry: ``(primitive, impl name) -> class``, plus reference aliases.

Parity: the mapping table in ``ddlb/benchmark.py:43-56``. The native slot replaces the
reference's nvFuser / TransformerEngine / JAX slots (SURVEY.md §7.1 slot mapping):

=====================  ============================================================
reference impl         here
=====================  ============================================================
compute_only           compute_only (``size``; + ``gemm``)           [also tp_rowwise]
pytorch                pytorch (RCCL + hipBLASLt vendor baseline)
fuser                  native (same option names; backend nccl->rccl, cuda->ipc)
transformer_engine     native ``algorithm=p2p_pipeline`` (TE userbuffers = ring-exchange
                       AG overlap, ``TPColumnwise/transformer_engine.py:51-72``)
jax                    native ``algorithm=default`` (XLA's all-gather + matmul)
=====================  ============================================================
"""

from __future__ import annotations

import importlib
from typing import Any, Dict, Tuple

_REGISTRY: Dict[str, Dict[str, Tuple[str, str]]] = {
    "tp_columnwise": {
        "compute_only": ("ddlb_amd.primitives.tp_columnwise.compute_only", "ComputeOnlyTPColumnwise"),
        "pytorch": ("ddlb_amd.primitives.tp_columnwise.pytorch", "PyTorchTPColumnwise"),
        "native": ("ddlb_amd.primitives.tp_columnwise.native", "NativeTPColumnwise"),
    },
    "tp_rowwise": {
        "compute_only": ("ddlb_amd.primitives.tp_rowwise.compute_only", "ComputeOnlyTPRowwise"),
        "pytorch": ("ddlb_amd.primitives.tp_rowwise.pytorch", "PyTorchTPRowwise"),
        "native": ("ddlb_amd.primitives.tp_rowwise.native", "NativeTPRowwise"),
    },
}

#: alias name -> (target impl, option overrides, note shown once)
_ALIASES: Dict[str, Tuple[str, Dict[str, Any], str]] = {
    "fuser": ("native", {}, "fuser (nvFuser) -> native MI355X implementation"),
    "transformer_engine": ("native", {"algorithm": "p2p_pipeline"},
                           "transformer_engine (userbuffers ring AG overlap) -> native p2p_pipeline"),
    "jax": ("native", {"algorithm": "default"}, "jax (XLA SPMD) -> native default"),
}


def implementations(primitive: str):
    if primitive not in _REGISTRY:
        raise ValueError(f"Unknown primitive: {primitive}")
    return sorted(_REGISTRY[primitive]) + sorted(_ALIASES)


def resolve(primitive: str, impl: str, options: Dict[str, Any]):
    """Return ``(cls, options, note)``; unknown option keys are dropped like the reference
    worker does (``ddlb/benchmark.py:76-77``)."""
    if primitive not in _REGISTRY:
        raise ValueError(f"Unknown primitive: {primitive}")
    note = ""
    opts = dict(options)
    if impl in _ALIASES:
        target, overrides, note = _ALIASES[impl]
        opts.update(overrides)
        impl = target
    if impl not in _REGISTRY[primitive]:
        raise ValueError(f"Unknown implementation '{impl}' for primitive '{primitive}'")
    module_path, cls_name = _REGISTRY[primitive][impl]
    cls = getattr(importlib.import_module(module_path), cls_name)
    defaults = getattr(cls, "DEFAULT_OPTIONS", {})
    opts = {k: v for k, v in opts.items() if k in defaults}
    return cls, opts, note
