"""The pt4 ablation lab stays applicable to the product kernel (CPU only, no compile).

`research/lab/pt4_ablate.py` times text-patched copies of `csrc/gemm/gemm_kernels.h`; a pattern
that no longer matches the product (the kernel moved on) must fail here, not on the GPU box in
the middle of a session (round 6: the store patches drifted when the C park landed).
"""

import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lab():
    spec = importlib.util.spec_from_file_location(
        "pt4_ablate", os.path.join(ROOT, "research", "lab", "pt4_ablate.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


LAB = _lab()


@pytest.mark.parametrize("variant", sorted(v for v in LAB.PATCHES if v != "ref"))
def test_variant_applies(variant):
    """Every pattern of the variant (or its diff) matches the product header exactly once."""
    text = LAB.patched_header(variant)
    product = LAB.source("gemm_kernels.h", "base")
    i = text.index("void gemm_tn_pt4_kernel(")
    assert "void gemm_tn_pt8_kernel(" in text[i:]
    if variant != "base":
        assert text != product, f"{variant} changed nothing"


def test_combination_variant_is_union():
    """A combination variant applies exactly its parts' patches."""
    combo = [v for v, p in LAB.PATCHES.items() if isinstance(p, str)]
    assert combo, "no combination variant"
    for v in combo:
        for part in LAB.PATCHES[v].split("+"):
            assert part in LAB.PATCHES and not isinstance(LAB.PATCHES[part], str)
