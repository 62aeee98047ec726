"""Build the native extension ``ddlb_amd/_C*.so`` in-tree with hipcc for gfx950.

No hipify, no ``torch.utils.cpp_extension`` (which hipifies CUDA sources): every source under
``csrc/`` is CDNA4 HIP / C++ and is compiled directly::

    python -m ddlb_amd._build            # incremental
    python -m ddlb_amd._build --force    # rebuild everything

The module links against the ROCm HIP runtime and RCCL by soname (``libamdhip64.so.7``,
``librccl.so.1``); ``ddlb_amd.ops`` imports torch first, so those sonames resolve to the copies
torch already loaded and the process keeps ONE HIP runtime and ONE RCCL.
"""

from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
PKG = os.path.join(ROOT, "ddlb_amd")
ARCH = os.environ.get("DDLB_OFFLOAD_ARCH", os.environ.get("PYTORCH_ROCM_ARCH", "gfx950"))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

SOURCES = [  # heaviest translation units first (the parallel build's critical path)
    "gemm/gemm_bf16_bf16.hip",
    "gemm/gemm_bf16_f32.hip",
    "gemm/gemm_fp8_bf16.hip",
    "gemm/gemm_fp8_f16.hip",
    "gemm/gemm_fp8_f32.hip",
    "gemm/gemm_f16_f16.hip",
    "gemm/gemm_f16_f32.hip",
    "gemm/gemm_f32_f32.hip",
    "gemm/gemm_mx.hip",
    "gemm/gemm_generic.hip",
    "gemm/gemm_mfma.hip",
    "runtime/kernels.hip",
    "comm/comm.cpp",
    "runtime/plan.cpp",
    "bindings.cpp",
]
HEADERS = ["gemm/gemm.h", "gemm/gemm_kernels.h", "gemm/gemm_entry.h", "gemm/tile_map.h",
           "runtime/kernels.h",
           "comm/comm.h", "runtime/plan.h", "runtime/plan_ir.h"]


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_C" + suffix)


def _hipcc() -> str:
    for cand in (os.path.join(ROCM, "bin", "hipcc"), shutil.which("hipcc") or ""):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm install expected under /opt/rocm)")


def _includes():
    import pybind11

    inc = [CSRC, sysconfig.get_paths()["include"], pybind11.get_include(),
           os.path.join(ROCM, "include")]
    try:  # only ATen/dlpack.h is used from torch's headers
        import importlib.util

        spec = importlib.util.find_spec("torch")
        if spec and spec.origin:
            inc.append(os.path.join(os.path.dirname(spec.origin), "include"))
    except Exception:
        pass
    return inc


def _torch_lib_dir() -> str:
    import importlib.util

    spec = importlib.util.find_spec("torch")
    return os.path.join(os.path.dirname(spec.origin), "lib") if spec and spec.origin else ""


def _digest(rels) -> str:
    import hashlib

    h = hashlib.sha256()
    for rel in rels:
        with open(os.path.join(CSRC, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    return h.hexdigest()


def _stamp_ok(path: str, digest: str) -> bool:
    stamp = path + ".sha256"
    if not (os.path.exists(path) and os.path.exists(stamp)):
        return False
    with open(stamp) as f:
        return f.read().strip() == digest


def _write_stamp(path: str, digest: str) -> None:
    with open(path + ".sha256", "w") as f:
        f.write(digest + "\n")


def _compile(src_rel: str, force: bool, verbose: bool):
    """-> (object path, recompiled?). An object is rebuilt when the digest of its source plus
    every header differs from the one recorded next to it (content, not file times)."""
    src = os.path.join(CSRC, src_rel)
    obj = os.path.join(BUILD, src_rel.replace("/", "_") + ".o")
    digest = _digest([src_rel] + HEADERS)
    if not force and _stamp_ok(obj, digest):
        return obj, False
    cmd = [_hipcc(), "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
           "-Wno-unused-result", "-DNDEBUG"]
    if src.endswith(".cpp"):
        cmd += ["-x", "hip"]  # host code that includes HIP headers; no device code inside
    cmd += [f"-I{d}" for d in _includes()] + ["-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src_rel}:\n{r.stderr[-6000:]}")
    _write_stamp(obj, digest)
    return obj, True


def source_digest() -> str:
    """sha256 over every source and header the extension is built from (in build order)."""
    return _digest(SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = False, jobs: int = 0) -> str:
    """Compile what changed and link ``ddlb_amd/_C*.so``. Objects and the .so carry the digest
    of the sources they were built from (``<file>.sha256``): whatever differs from the tree's
    content is rebuilt, so a checkout or copy that resets file times cannot leave a stale .so."""
    os.makedirs(BUILD, exist_ok=True)
    out = ext_path()
    digest = source_digest()
    jobs = jobs or min(len(SOURCES), max(1, os.cpu_count() or 4), 8)
    with ThreadPoolExecutor(jobs) as ex:
        res = list(ex.map(lambda s: _compile(s, force, verbose), SOURCES))
    objs = [o for o, _ in res]
    if not any(rebuilt for _, rebuilt in res) and _stamp_ok(out, digest):
        return out
    tl = _torch_lib_dir()
    cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", out + ".tmp",
           f"-L{ROCM}/lib", "-lrccl", "-lamdhip64"]
    if tl:
        cmd.append(f"-Wl,-rpath,{tl}")
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    os.replace(out + ".tmp", out)
    _write_stamp(out, digest)
    return out


def main(argv=None) -> None:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--force", action="store_true")
    p.add_argument("-v", "--verbose", action="store_true")
    p.add_argument("-j", "--jobs", type=int, default=0)
    a = p.parse_args(argv)
    print(build(force=a.force, verbose=a.verbose, jobs=a.jobs))


if __name__ == "__main__":
    main(sys.argv[1:])
