"""TP-Rowwise primitive: K-sharded GEMM followed by a sequence-parallel reduce-scatter.

Parity: ``ddlb/primitives/TPRowwise/tp_rowwise.py:13-185``.

Rank ``r`` holds ``A[:, r*k/d:(r+1)*k/d]`` (``[m, k/d]``) and ``B[r*k/d:(r+1)*k/d, :]``
(``[k/d, n]``). Its result is row block ``r`` of ``A @ B``: ``[m/d, n]``, i.e. the partial
products summed over ranks and scattered along M (SURVEY.md §2.6 "Row default").
"""

from __future__ import annotations

from ddlb_amd.primitives.base import Primitive, uniform_pm1


class TPRowwise(Primitive):
    NAME = "tp_rowwise"

    def _check_shape(self) -> None:
        d = self.world_size
        if self.k % d != 0:
            raise ValueError(f"Matrix dimension k ({self.k}) must be divisible by world_size ({d})")
        if self.m % d != 0:
            raise ValueError(f"Matrix dimension m ({self.m}) must be divisible by world_size ({d})")

    @property
    def m_local(self) -> int:
        return self.m // self.world_size

    @property
    def k_local(self) -> int:
        return self.k // self.world_size

    def _input_setup(self) -> None:
        g, dev = self._generator, self.device
        self.A_unsharded = uniform_pm1((self.m, self.k), self.dtype, g, dev)
        self.B_unsharded = uniform_pm1((self.k, self.n), self.dtype, g, dev)
        k0 = self.rank * self.k_local
        self.A = self.A_unsharded[:, k0:k0 + self.k_local].contiguous()
        self.B = self.B_unsharded[k0:k0 + self.k_local].contiguous()

    def expected(self):
        full = self._ref_matmul(self.A_unsharded, self.B_unsharded)
        r0 = self.rank * self.m_local
        return full[r0:r0 + self.m_local]
