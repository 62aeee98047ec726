"""native TP-Columnwise: HIP MFMA GEMM + RCCL / IPC all-gather, overlapped by a C++ plan executor.

Replaces the reference's ``fuser`` (nvFuser), ``transformer_engine`` and ``jax`` slots
(``ddlb/primitives/TPColumnwise/fuser.py``, ``transformer_engine.py``, ``jax_tp.py``); options in
:mod:`ddlb_amd.primitives.native_common`, algorithms in :mod:`ddlb_amd.parallel.algorithms`.

The activation shard lives in this rank's slot of the symmetric gather buffer (in-place
all-gather, zero-copy input): ``self.A`` is copied there once at construction. ``input_copy=True``
re-copies it at the start of every ``run()`` instead, for a producer that cannot write in place.
The weight is stored ``[n, k]`` (K-contiguous), like ``te.Linear``.
"""

from __future__ import annotations

from ddlb_amd.parallel.algorithms import build_tp_columnwise
from ddlb_amd.primitives.native_common import (COMMON_ALIASES, COMMON_ALLOWED, COMMON_DEFAULTS,
                                               algo_config, dtype_codes, maybe_enable_graph,
                                               share_cus)
from ddlb_amd.primitives.tp_columnwise.base import TPColumnwise


class NativeTPColumnwise(TPColumnwise):
    DEFAULT_OPTIONS = {**{k: v for k, v in COMMON_DEFAULTS.items() if k in ("backend",)},
                       "order": "AG_before",
                       **{k: v for k, v in COMMON_DEFAULTS.items() if k != "backend"},
                       "input_copy": False}
    ALLOWED_VALUES = {**COMMON_ALLOWED, "order": ["AG_before", "AG_after"],
                      "input_copy": [True, False]}
    OPTION_ALIASES = COMMON_ALIASES

    def __init__(self, *args, **kwargs):
        import torch

        super().__init__(*args, **kwargs)
        if not self.communicator.is_gpu:
            raise RuntimeError("the native implementation needs a ROCm GPU (use compute_only / "
                               "pytorch on the CPU)")
        self.cfg = share_cus(algo_config(self.options, order=self.options["order"]),
                             self.communicator)
        din, dout = dtype_codes(self.dtype)
        self.plan, self.io = build_tp_columnwise(self.rank, self.world_size, self.m, self.n,
                                                 self.k, din, dout, self.cfg)
        self.ctx = self.communicator.native()
        self.bound = self.ctx.bind(self.plan, trace=bool(self.options["trace"]))
        self.graph = maybe_enable_graph(self.bound, self.options["graph"])
        self.a_slot = self.bound.view(self.io.a)
        self.a_slot.copy_(self.A)
        self.bound.view(self.io.b).copy_(self.B.t())
        self.out = self.bound.view(self.io.out)
        self._input_copy = bool(self.options["input_copy"])
        torch.cuda.synchronize()
        self.communicator.barrier()

    def run(self):
        if self._input_copy:
            self.a_slot.copy_(self.A, non_blocking=True)
        self.bound.run()
        return self.out

    def check_health(self) -> None:
        self.bound.check_health()

    def validate(self, result) -> None:
        self.check_health()
        super().validate(result)

    def close(self) -> None:
        if getattr(self, "bound", None) is not None:
            self.bound.close()
            self.bound = None
