"""Model-level building blocks on top of the primitives.

* :mod:`ddlb_amd.models.shapes`  — TP GEMM shapes of real transformer layers (Llama 3, GPT-3,
  Qwen2, Mixtral) -> benchmark sweeps (``python -m ddlb_amd.models``).
* :mod:`ddlb_amd.models.tp_mlp`  — sequence-parallel TP MLP block (AG+GEMM+act -> GEMM+RS).
"""

from ddlb_amd.models.shapes import MODELS, LayerGemm, ModelSpec, benchmark_configs, layer_gemms

__all__ = ["MODELS", "ModelSpec", "LayerGemm", "layer_gemms", "benchmark_configs"]
