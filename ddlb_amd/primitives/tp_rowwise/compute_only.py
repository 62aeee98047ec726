"""compute_only TP-Rowwise: the K-sharded partial GEMM alone (no reduce-scatter).

Not present in the reference (``ddlb/benchmark.py:51-55`` registers none for tp_rowwise); added
so the GEMM share of the rowwise pipelines can be measured on its own. ``size=sharded`` runs
``[m, k/d] x [k/d, n]`` (this rank's real work); ``unsharded`` runs the full ``[m, k] x [k, n]``.
Validation compares against the matching fp32 product.
"""

from __future__ import annotations

from ddlb_amd.primitives.gemm_select import GemmBackend
from ddlb_amd.primitives.tp_rowwise.base import TPRowwise


class ComputeOnlyTPRowwise(TPRowwise):
    DEFAULT_OPTIONS = {"size": "sharded", "gemm": "auto"}
    ALLOWED_VALUES = {"size": ["sharded", "unsharded"], "gemm": ["auto", "hip", "torch", "torch_nt"]}

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.size = self.options["size"]
        self.gemm = GemmBackend(self.options["gemm"], self.device, self.dtype)
        if self.size == "unsharded":
            self.a_in, b = self.A_unsharded, self.B_unsharded
        else:
            self.a_in, b = self.A, self.B
        self._b_ref = b
        self.w = self.gemm.prepare_weight(b)
        self.out = self.gemm.alloc_out(self.m, self.n)

    def run(self):
        return self.gemm(self.a_in, self.w, self.out)

    def expected(self):
        return self._ref_matmul(self.a_in, self._b_ref)
