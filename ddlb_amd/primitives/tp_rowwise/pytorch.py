"""pytorch TP-Rowwise: ``torch.matmul`` (hipBLASLt) + ``reduce_scatter_tensor`` (RCCL).

Parity: ``ddlb/primitives/TPRowwise/pytorch.py:13-86``. The partial ``[m, n]`` product of the
local K slice is reduce-scattered along M, so rank ``r`` ends with row block ``r``.
Options as in the columnwise pytorch slot (``backend``, ``empty_cache``).
"""

from __future__ import annotations

from ddlb_amd.primitives.backends import UCC_BACKENDS, VendorMatmul, reduce_scatter_into, \
    resolve_torch_backend
from ddlb_amd.primitives.tp_rowwise.base import TPRowwise


class PyTorchTPRowwise(TPRowwise):
    DEFAULT_OPTIONS = {"backend": "nccl", "empty_cache": True}
    ALLOWED_VALUES = {"backend": ["nccl", "rccl", "gloo", *UCC_BACKENDS],
                      "empty_cache": [True, False]}

    def __init__(self, *args, **kwargs):
        import torch

        super().__init__(*args, **kwargs)
        resolve_torch_backend(self.options["backend"], self.communicator)
        self.communicator.ensure_process_group()
        self._empty_cache = bool(self.options["empty_cache"]) and self.communicator.is_gpu
        self.mm = VendorMatmul(self.B, self.out_dtype)
        self.result_shard = torch.empty((self.m_local, self.n), dtype=self.out_dtype,
                                        device=self.device)

    def run(self):
        import torch

        if self._empty_cache:
            torch.cuda.empty_cache()
        local = self.mm(self.A)
        reduce_scatter_into(self.result_shard, local)
        return self.result_shard
