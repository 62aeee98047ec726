"""Host-side native tests: C++ checks of the GEMM's index maps (csrc/gemm/tile_map.h) compiled for
the host only with AddressSanitizer + UndefinedBehaviorSanitizer (GPU-side
sanitizers are not available on MI355X here, so every map the kernels use is also a host
function and is checked here for bijectivity / coverage)."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None,
                    reason="hipcc not installed")
def test_tile_maps_host_asan_ubsan(tmp_path):
    hipcc = HIPCC if os.path.exists(HIPCC) else shutil.which("hipcc")
    exe = str(tmp_path / "tile_maps")
    cmd = [hipcc, "-x", "hip", "--cuda-host-only", "-std=c++17", "-O1", "-g",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-fno-omit-frame-pointer", f"-I{os.path.join(ROOT, 'csrc')}",
           os.path.join(ROOT, "tests", "native", "test_tile_maps.cpp"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    # verify_asan_link_order=0: the process environment may preload other libraries; the
    # sanitizer runtime is linked into the test binary itself
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "tile maps ok" in r.stdout


def test_op_word_layout_matches_native():
    """The Python plan encoder and the C++ executor agree on the op size (csrc/runtime/plan.h
    kOpWords); a mismatch would shift every op's fields. Skipped when the extension is not built."""
    import glob
    import importlib

    if not glob.glob(os.path.join(ROOT, "ddlb_amd", "_C*.so")):
        pytest.skip("native extension not built")
    import torch  # noqa: F401  (shared HIP runtime first)

    from ddlb_amd.parallel.plan import OP_WORDS

    C = importlib.import_module("ddlb_amd._C")
    assert C.OP_WORDS == OP_WORDS
