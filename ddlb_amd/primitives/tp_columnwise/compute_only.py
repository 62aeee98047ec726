"""compute_only TP-Columnwise: the GEMM alone, no communication.

Parity: ``ddlb/primitives/TPColumnwise/compute_only.py:8-55`` (option ``size``).
Added option ``gemm``: ``hip`` = our MFMA kernel (weight stored ``[n, k]``), ``torch`` =
``torch.matmul`` (hipBLASLt on GPU, the only choice on CPU), ``auto`` = hip on GPU.

Unlike the reference, ``size=sharded`` is validated too (against the local rows) instead of
being skipped (``compute_only.py:52-53``). Its TFLOPS keeps the reference's ``2*m*n*k``
numerator, which over-counts by ``d`` — kept for comparability.
"""

from __future__ import annotations

from ddlb_amd.primitives.tp_columnwise.base import TPColumnwise
from ddlb_amd.primitives.gemm_select import GemmBackend


class ComputeOnlyTPColumnwise(TPColumnwise):
    DEFAULT_OPTIONS = {"size": "sharded", "gemm": "auto"}
    ALLOWED_VALUES = {"size": ["sharded", "unsharded"], "gemm": ["auto", "hip", "torch", "torch_nt"]}

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.size = self.options["size"]
        self.a_in = self.A_unsharded if self.size == "unsharded" else self.A
        self.gemm = GemmBackend(self.options["gemm"], self.device, self.dtype)
        self.w = self.gemm.prepare_weight(self.B)
        self.out = self.gemm.alloc_out(self.a_in.shape[0], self.n)

    def run(self):
        return self.gemm(self.a_in, self.w, self.out)

    def expected(self):
        if self.size == "unsharded":
            return self._ref_matmul(self.A_unsharded, self.B)
        return self._ref_matmul(self.A, self.B)
