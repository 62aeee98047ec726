"""TP-Columnwise primitive: sequence-sharded all-gather of A followed by a GEMM.

Parity: ``ddlb/primitives/TPColumnwise/tp_columnwise.py:13-162``.

Each rank holds ``A_r = A[r*m/d:(r+1)*m/d, :]`` (``[m/d, k]``, the sequence shard) and the full
local weight block ``B`` (``[k, n]``, identical on every rank). The result on every rank is
``C = A @ B`` (``[m, n]``), gathered rows in rank-major order.
"""

from __future__ import annotations

from ddlb_amd.primitives.base import Primitive, uniform_pm1


class TPColumnwise(Primitive):
    NAME = "tp_columnwise"

    def _check_shape(self) -> None:
        if self.m % self.world_size != 0:
            raise ValueError(f"Matrix dimension m ({self.m}) must be divisible by world_size "
                             f"({self.world_size})")

    @property
    def m_local(self) -> int:
        return self.m // self.world_size

    def _input_setup(self) -> None:
        g, dev = self._generator, self.device
        self.A_unsharded = uniform_pm1((self.m, self.k), self.dtype, g, dev)
        r0 = self.rank * self.m_local
        self.A = self.A_unsharded[r0:r0 + self.m_local]
        self.B = uniform_pm1((self.k, self.n), self.dtype, g, dev)

    def expected(self):
        return self._ref_matmul(self.A_unsharded, self.B)
