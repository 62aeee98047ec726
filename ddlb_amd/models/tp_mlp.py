"""Sequence-parallel tensor-parallel MLP block built from the two primitives (Megatron-style).

Per rank r of d:   X_r [S/d, H]  (sequence shard)
    H1  = act( AllGather_S(X) @ W1[:, r-th F/d block] )          tp_columnwise, fused epilogue act
    Y_r = ReduceScatter_S( H1 @ W2[r-th F/d block, :] )           tp_rowwise
so Y_r = rows r*S/d.. of act(X @ W1) @ W2. The columnwise output buffer is bound as the rowwise
input (zero copy), the activation runs inside the first GEMM's epilogue, and both plans are
enqueued on the caller's stream: one forward = two native calls.

This is what the two DDLB primitives exist for (a TP+SP transformer MLP); the reference benchmarks
them only in isolation.
"""

from __future__ import annotations

from typing import Dict, Optional

from ddlb_amd.parallel.algorithms import AlgoConfig, build_tp_columnwise, build_tp_rowwise
from ddlb_amd.parallel.plan import ACT_CODE, NAME_DT


class SequenceParallelMLP:
    def __init__(self, hidden: int, ffn: int, seq: int, dtype: str = "bfloat16",
                 act: str = "gelu", col: Optional[Dict] = None, row: Optional[Dict] = None,
                 seed: int = 0):
        import torch

        from ddlb_amd.communicator import Communicator
        from ddlb_amd.primitives.base import uniform_pm1

        self.comm = Communicator()
        self.comm.ensure_process_group()
        d, r = self.comm.world_size, self.comm.rank
        if ffn % d or seq % d:
            raise ValueError("ffn and seq must be divisible by the world size")
        self.H, self.F, self.S, self.d, self.r = hidden, ffn, seq, d, r
        self.dtype, self.act = dtype, act
        dev = self.comm.device
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        scale1, scale2 = hidden ** -0.5, ffn ** -0.5
        self.X_full = uniform_pm1((seq, hidden), dtype, g, dev)
        self.W1 = (uniform_pm1((hidden, ffn), "float32", g, dev) * scale1).to(self.X_full.dtype)
        self.W2 = (uniform_pm1((ffn, hidden), "float32", g, dev) * scale2).to(self.X_full.dtype)
        fl = ffn // d
        self.w1_r = self.W1[:, r * fl:(r + 1) * fl]
        self.w2_r = self.W2[r * fl:(r + 1) * fl]
        din = NAME_DT[dtype]
        ccfg = AlgoConfig(**{**dict(algorithm="coll_pipeline", backend="rccl", s=4), **(col or {}),
                             "act": ACT_CODE[act]})
        rcfg = AlgoConfig(**{**dict(algorithm="coll_pipeline", backend="rccl", s=4),
                             **(row or {})})
        self.col_plan, self.col_io = build_tp_columnwise(r, d, seq, fl, hidden, din, din, ccfg)
        self.row_plan, self.row_io = build_tp_rowwise(r, d, seq, hidden, ffn, din, din, rcfg)
        if not self.comm.is_gpu:
            raise RuntimeError("SequenceParallelMLP runs the native plans: it needs a ROCm GPU")
        ctx = self.comm.native()
        self.col = ctx.bind(self.col_plan)
        h1 = self.col.view(self.col_io.out)          # [S, F/d]
        self.row = ctx.bind(self.row_plan, externals={self.row_io.a.buf: h1})
        sl = seq // d
        self.col.view(self.col_io.a).copy_(self.X_full[r * sl:(r + 1) * sl])
        self.col.view(self.col_io.b).copy_(self.w1_r.t())
        self.row.view(self.row_io.b).copy_(self.w2_r.t())
        self.out = self.row.view(self.row_io.out)    # [S/d, H]
        torch.cuda.synchronize()
        self.comm.barrier()

    @property
    def flops(self) -> float:
        """Whole-job FLOPs of one forward: 2*S*H*F for each of the two GEMMs."""
        return 4.0 * self.S * self.H * self.F

    def forward(self):
        self.col.run()
        self.row.run()
        return self.out

    def reference(self):
        import torch

        from ddlb_amd.parallel.sim import apply_act

        h = apply_act(self.X_full.float() @ self.W1.float(), ACT_CODE[self.act])
        h = h.to(self.X_full.dtype).float()   # the block materialises H1 in the compute dtype
        y = h @ self.W2.float()
        sl = self.S // self.d
        return y[self.r * sl:(self.r + 1) * sl]

    def validate(self, out=None) -> None:
        import torch

        out = self.out if out is None else out
        torch.testing.assert_close(out.float(), self.reference(), rtol=0.03, atol=0.03)

    def close(self) -> None:
        self.row.close()
        self.col.close()
