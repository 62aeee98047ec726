"""Backend-name handling and thin torch.distributed helpers shared by the implementations.

The reference accepts ``nccl``, ``ucc``, ``ucc/tl/{nccl,cuda,ucp}`` and (nvFuser) ``cuda``
(``ddlb/primitives/TPColumnwise/pytorch.py:31``, ``fuser.py:171``). On MI355X:

* ``nccl`` / ``rccl``      -> RCCL (torch's ``"nccl"`` backend on ROCm is RCCL);
* ``cuda`` / ``ipc``       -> HIP IPC symmetric memory over xGMI (native slot only);
* ``ucc`` / ``ucc/tl/*``   -> rejected: UCC/UCX are not part of this stack.
"""

from __future__ import annotations

UCC_BACKENDS = ("ucc", "ucc/tl/nccl", "ucc/tl/cuda", "ucc/tl/ucp")


class BackendUnavailable(ValueError):
    pass


def resolve_torch_backend(name: str, communicator) -> str:
    """Map a reference backend name to the torch.distributed backend this stack uses."""
    if name in UCC_BACKENDS:
        raise BackendUnavailable(
            f"backend '{name}' needs UCC/UCX, which the MI355X stack does not ship; "
            "use backend=nccl (RCCL over xGMI) or the native slot's backend=ipc")
    if name == "gloo":
        if communicator.is_gpu:
            raise BackendUnavailable("backend 'gloo' is CPU-only here; use nccl/rccl on GPU")
        return "gloo"
    if name in ("nccl", "rccl"):
        return communicator.backend  # RCCL on GPU, gloo when running the CPU plumbing path
    raise BackendUnavailable(f"unknown backend '{name}'")


def all_gather_into(out, inp) -> None:
    """``all_gather_into_tensor`` along dim 0; fp8 tensors travel as bytes."""
    import torch
    import torch.distributed as dist

    if inp.dtype == torch.float8_e4m3fn:
        out, inp = out.view(torch.uint8), inp.view(torch.uint8)
    inp = inp.contiguous()
    if dist.get_backend() == "gloo":
        parts = list(out.chunk(dist.get_world_size()))
        dist.all_gather(parts, inp)
        return
    dist.all_gather_into_tensor(out, inp)


def reduce_scatter_into(out, inp) -> None:
    """``reduce_scatter_tensor`` (SUM) along dim 0."""
    import torch.distributed as dist

    inp = inp.contiguous()
    if dist.get_backend() == "gloo":
        # gloo lacks reduce_scatter: all_reduce then take this rank's block
        tmp = inp.clone()
        dist.all_reduce(tmp)
        out.copy_(tmp.chunk(dist.get_world_size())[dist.get_rank()])
        return
    dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM)


class VendorMatmul:
    """``x @ B`` through the vendor library (hipBLASLt on GPU); fp8 via ``torch._scaled_mm``."""

    def __init__(self, b, out_dtype):
        import torch

        self.out_dtype = out_dtype
        self.fp8 = b.dtype == torch.float8_e4m3fn
        self.b = b
        self.scaled = False
        if self.fp8:
            self.b_col = b.t().contiguous().t()  # column-major, as _scaled_mm wants
            self.one = torch.ones((), dtype=torch.float32, device=b.device)
            self.b16 = b.to(torch.bfloat16)
            if b.is_cuda and hasattr(torch, "_scaled_mm"):
                try:
                    x = torch.zeros((16, b.shape[0]), dtype=b.dtype, device=b.device)
                    torch._scaled_mm(x, self.b_col, scale_a=self.one, scale_b=self.one,
                                     out_dtype=out_dtype)
                    self.scaled = True
                except Exception:
                    self.scaled = False

    def __call__(self, a):
        import torch

        if not self.fp8:
            return torch.matmul(a, self.b)
        if self.scaled:
            return torch._scaled_mm(a, self.b_col, scale_a=self.one, scale_b=self.one,
                                    out_dtype=self.out_dtype)
        return torch.matmul(a.to(torch.bfloat16), self.b16)
