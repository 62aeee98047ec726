"""ddlb_amd — MI355X-native distributed-GEMM benchmark framework.

Same capabilities and CLI/JSON/CSV surface as DDLB (samnordmann/ddlb), re-designed for
AMD Instinct MI355X (gfx950): hand-written CDNA4 MFMA GEMM kernels, RCCL over xGMI and HIP IPC
symmetric memory, a native C++ plan executor for the comm/compute-overlap pipelines, roctx /
rocprofv3 profiling hooks.

Heavy (torch / HIP) imports are deferred, as in the reference (``ddlb/__init__.py:7-30``), so the
parent runner process never creates a GPU context.
"""

__version__ = "0.1.0"

_LAZY = {
    "PrimitiveBenchmarkRunner": ("ddlb_amd.benchmark", "PrimitiveBenchmarkRunner"),
    "run_benchmark": ("ddlb_amd.cli.benchmark", "run_benchmark"),
    "TPColumnwise": ("ddlb_amd.primitives.tp_columnwise.base", "TPColumnwise"),
    "TPRowwise": ("ddlb_amd.primitives.tp_rowwise.base", "TPRowwise"),
    "ComputeOnlyTPColumnwise": ("ddlb_amd.primitives.tp_columnwise.compute_only",
                                "ComputeOnlyTPColumnwise"),
    "PyTorchTPColumnwise": ("ddlb_amd.primitives.tp_columnwise.pytorch", "PyTorchTPColumnwise"),
    "NativeTPColumnwise": ("ddlb_amd.primitives.tp_columnwise.native", "NativeTPColumnwise"),
    "ComputeOnlyTPRowwise": ("ddlb_amd.primitives.tp_rowwise.compute_only", "ComputeOnlyTPRowwise"),
    "PyTorchTPRowwise": ("ddlb_amd.primitives.tp_rowwise.pytorch", "PyTorchTPRowwise"),
    "NativeTPRowwise": ("ddlb_amd.primitives.tp_rowwise.native", "NativeTPRowwise"),
    "Communicator": ("ddlb_amd.communicator", "Communicator"),
}

__all__ = ["__version__", *_LAZY]


def __getattr__(name):
    if name in _LAZY:
        import importlib

        mod, attr = _LAZY[name]
        return getattr(importlib.import_module(mod), attr)
    raise AttributeError(f"module 'ddlb_amd' has no attribute {name!r}")
