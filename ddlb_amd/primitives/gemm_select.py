"""Select and drive the local GEMM used by the compute_only / pytorch / native slots.

``hip``   : our CDNA4 MFMA kernels (:mod:`ddlb_amd.ops.gemm`); weights are stored ``[n, k]``
            (K-contiguous, the layout both MFMA operands want — the same layout
            ``te.Linear`` keeps its weight in).
``torch`` : ``torch.matmul`` (hipBLASLt / rocBLAS on GPU, ATen on CPU) — the vendor baseline, with
            the reference's ``[k, n]`` weight (``TPColumnwise/pytorch.py:97``).
``torch_nt``: ``F.linear`` on the ``[n, k]`` weight — hipBLASLt's fastest layout (the one our
            kernels use), so the vendor comparison is like for like.
``auto``  : ``hip`` on a GPU, ``torch`` on the CPU. On a GPU ``auto`` never silently falls back:
            a missing extension raises (the driver checks the native library really ran).
"""

from __future__ import annotations

from ddlb_amd.primitives.base import output_dtype


class GemmBackend:
    def __init__(self, choice: str, device, dtype_name: str):
        self.device = device
        self.dtype_name = dtype_name
        self.out_dtype = output_dtype(dtype_name)
        if choice == "auto":
            choice = "hip" if device.type == "cuda" else "torch"
        if choice == "hip" and device.type != "cuda":
            raise RuntimeError("gemm=hip needs a ROCm GPU; use gemm=torch on the CPU")
        self.choice = choice
        if choice == "hip":
            from ddlb_amd.ops import gemm as _g

            _g.check_supported(dtype_name)
            self._hip = _g

    def prepare_weight(self, b):
        """``b`` is ``[k, n]``; the HIP kernel (and F.linear) consume ``[n, k]``."""
        if self.choice in ("hip", "torch_nt"):
            return b.t().contiguous()
        return b

    def alloc_out(self, rows: int, cols: int):
        import torch

        return torch.empty((rows, cols), dtype=self.out_dtype, device=self.device)

    def __call__(self, a, w, out=None):
        if self.choice == "hip":
            return self._hip.gemm(a, w, out=out)
        import torch

        if a.dtype == torch.float8_e4m3fn:
            a, w = a.to(torch.bfloat16), w.to(torch.bfloat16)
        if self.choice == "torch_nt":
            return torch.nn.functional.linear(a, w)
        if out is not None:
            return torch.matmul(a, w, out=out)
        return torch.matmul(a, w)
