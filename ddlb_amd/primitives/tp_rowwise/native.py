"""native TP-Rowwise: HIP MFMA GEMM + RCCL / IPC reduce-scatter, overlapped by the plan executor.

Replaces the reference's ``fuser`` and ``transformer_engine`` rowwise slots
(``ddlb/primitives/TPRowwise/fuser.py``, ``transformer_engine.py``). Every algorithm produces the
canonical contiguous output block ``r``. IPC reductions sum the d partials in f32
in one kernel and round once (RCCL's reduce-scatter sums in the wire dtype).
"""

from __future__ import annotations

from ddlb_amd.parallel.algorithms import build_tp_rowwise
from ddlb_amd.primitives.native_common import (COMMON_ALIASES, COMMON_ALLOWED, COMMON_DEFAULTS,
                                               algo_config, dtype_codes, maybe_enable_graph)
from ddlb_amd.primitives.tp_rowwise.base import TPRowwise


class NativeTPRowwise(TPRowwise):
    DEFAULT_OPTIONS = dict(COMMON_DEFAULTS)
    ALLOWED_VALUES = dict(COMMON_ALLOWED)
    OPTION_ALIASES = COMMON_ALIASES

    def __init__(self, *args, **kwargs):
        import torch

        super().__init__(*args, **kwargs)
        if not self.communicator.is_gpu:
            raise RuntimeError("the native implementation needs a ROCm GPU")
        opts = self.options
        if opts["algorithm"] == "p2p_pipeline" and int(opts["s"]) != self.world_size:
            opts.options["s"] = self.world_size  # reference forces s = d (TPRowwise/fuser.py:256)
        self.cfg = algo_config(opts)
        din, dout = dtype_codes(self.dtype)
        self.plan, self.io = build_tp_rowwise(self.rank, self.world_size, self.m, self.n, self.k,
                                              din, dout, self.cfg)
        self.ctx = self.communicator.native()
        self.bound = self.ctx.bind(self.plan, trace=bool(self.options["trace"]))
        self.graph = maybe_enable_graph(self.bound, self.options["graph"])
        self.bound.view(self.io.a).copy_(self.A)
        self.bound.view(self.io.b).copy_(self.B.t())
        self.out = self.bound.view(self.io.out)
        torch.cuda.synchronize()
        self.communicator.barrier()

    def run(self):
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
