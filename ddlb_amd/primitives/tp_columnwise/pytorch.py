"""pytorch TP-Columnwise: ``torch.distributed`` all-gather (RCCL) + ``torch.matmul`` (hipBLASLt).

Parity: ``ddlb/primitives/TPColumnwise/pytorch.py:13-105`` — the vendor-library baseline the
native slot is measured against. ``order=AG_before`` gathers A then multiplies; ``AG_after``
multiplies the local shard and gathers C.

* ``backend``: ``nccl`` and ``rccl`` both mean RCCL (torch's ``"nccl"`` backend on ROCm);
  ``gloo`` is allowed on the CPU. UCC/UCX transports do not exist on this platform and are
  rejected with an explicit error.
* ``empty_cache``: the reference calls ``torch.cuda.empty_cache()`` inside every timed
  ``run()`` (``pytorch.py:92``); kept ON by default for parity, switch off to time the
  collective + GEMM alone.
* fp8 (e4m3) uses ``torch._scaled_mm`` (hipBLASLt fp8) with unit scales when available.
"""

from __future__ import annotations

from ddlb_amd.primitives.backends import UCC_BACKENDS, VendorMatmul, all_gather_into, \
    resolve_torch_backend
from ddlb_amd.primitives.tp_columnwise.base import TPColumnwise


class PyTorchTPColumnwise(TPColumnwise):
    DEFAULT_OPTIONS = {"backend": "nccl", "order": "AG_before", "empty_cache": True}
    ALLOWED_VALUES = {"backend": ["nccl", "rccl", "gloo", *UCC_BACKENDS],
                      "order": ["AG_before", "AG_after"],
                      "empty_cache": [True, False]}

    def __init__(self, *args, **kwargs):
        import torch

        super().__init__(*args, **kwargs)
        resolve_torch_backend(self.options["backend"], self.communicator)
        self.communicator.ensure_process_group()
        self.order = self.options["order"]
        self._empty_cache = bool(self.options["empty_cache"]) and self.communicator.is_gpu
        self.mm = VendorMatmul(self.B, self.out_dtype)
        if self.order == "AG_before":
            self.A_gathered = torch.empty((self.m, self.k), dtype=self.A.dtype, device=self.device)
        else:
            self.result_gathered = torch.empty((self.m, self.n), dtype=self.out_dtype,
                                               device=self.device)

    def run(self):
        import torch

        if self._empty_cache:
            torch.cuda.empty_cache()
        if self.order == "AG_before":
            all_gather_into(self.A_gathered, self.A)
            return self.mm(self.A_gathered)
        local = self.mm(self.A)
        all_gather_into(self.result_gathered, local)
        return self.result_gathered
