"""CLI / programmatic entry points (parity: ``ddlb/cli/__init__.py:1-5``)."""

from ddlb_amd.cli.benchmark import main, run_benchmark

__all__ = ["run_benchmark", "main"]
