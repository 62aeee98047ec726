"""Distributed-GEMM primitives (parity: ``ddlb/primitives/__init__.py``). Lazy exports."""

from ddlb_amd.primitives.registry import implementations, resolve

__all__ = ["implementations", "resolve"]
