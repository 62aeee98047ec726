"""roctx markers and the rocprofv3 capture window.

Parity: the reference brackets 5 ``run()`` calls with ``cudaProfilerStart/Stop`` so
``nsys --capture-range=cudaProfilerApi`` records one window per benchmark row
(``ddlb/benchmark.py:89-104``). Here the same window is delimited with
``roctxProfilerResume(0)`` / ``roctxProfilerPause(0)`` for ``rocprofv3 --selected-regions``
and every profiled ``run()`` gets a ``roctxRangePush("<impl>")`` range, e.g.::

    rocprofv3 --selected-regions --kernel-trace --marker-trace --stats -d gpurun_out/prof \
        -- python -m ddlb_amd --primitive tp_columnwise -m 65536 -n 1024 -k 1024 --impl native

The library is loaded with ``ctypes`` from the ROCm install; when it is absent every call is
a no-op (CPU CI).
"""

from __future__ import annotations

import ctypes
import os
from contextlib import contextmanager

_LIB = None
_TRIED = False
_CANDIDATES = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
               "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", "libroctx64.so.4", "libroctx64.so")


def _lib():
    global _LIB, _TRIED
    if _TRIED:
        return _LIB
    _TRIED = True
    if os.environ.get("DDLB_ROCTX", "1") == "0":
        return None
    for name in _CANDIDATES:
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _LIB = lib
            break
        except (OSError, AttributeError):
            continue
    return _LIB


def available() -> bool:
    return _lib() is not None


def range_push(name: str) -> None:
    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())


def range_pop() -> None:
    lib = _lib()
    if lib is not None:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _lib()
    if lib is not None:
        lib.roctxMarkA(name.encode())


@contextmanager
def roctx_range(name: str):
    range_push(name)
    try:
        yield
    finally:
        range_pop()


def profiler_resume() -> None:
    """Open the rocprofv3 ``--selected-regions`` capture window (cudaProfilerStart analogue)."""
    lib = _lib()
    if lib is None:
        return
    fn = getattr(lib, "roctxProfilerResume", None)
    if fn is not None:
        fn(ctypes.c_uint64(0))


def profiler_pause() -> None:
    lib = _lib()
    if lib is None:
        return
    fn = getattr(lib, "roctxProfilerPause", None)
    if fn is not None:
        fn(ctypes.c_uint64(0))
