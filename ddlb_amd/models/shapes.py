"""Tensor-parallel GEMM shapes of real transformer layers.

A DDLB sweep is a grid of (m, n, k). What a user actually wants to know is how the TP GEMMs of
*their* model behave at *their* TP degree and token count. This catalog maps a model + TP degree +
tokens-per-step to the four sequence-parallel TP GEMMs of one transformer layer, in this
framework's conventions:

* ``tp_columnwise`` (AG -> GEMM): m = tokens, n = the per-rank output width (N_total / tp),
  k = hidden — QKV projection and MLP up(+gate) projection;
* ``tp_rowwise`` (GEMM -> RS): m = tokens, n = hidden, k = the full contraction (sharded inside) —
  attention output projection and MLP down projection.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Tuple


@dataclass(frozen=True)
class ModelSpec:
    name: str
    hidden: int
    ffn: int
    heads: int
    kv_heads: int
    head_dim: int
    layers: int
    gated_mlp: bool = True   # SwiGLU-style: up and gate projections fused into one GEMM


MODELS: Dict[str, ModelSpec] = {m.name: m for m in [
    ModelSpec("llama3-8b", 4096, 14336, 32, 8, 128, 32),
    ModelSpec("llama3-70b", 8192, 28672, 64, 8, 128, 80),
    ModelSpec("llama3-405b", 16384, 53248, 128, 8, 128, 126),
    ModelSpec("mixtral-8x7b-expert", 4096, 14336, 32, 8, 128, 32),
    ModelSpec("gpt3-175b", 12288, 49152, 96, 96, 128, 96, gated_mlp=False),
    ModelSpec("qwen2-72b", 8192, 29568, 64, 8, 128, 80),
]}


@dataclass(frozen=True)
class LayerGemm:
    name: str
    primitive: str
    m: int
    n: int
    k: int

    @property
    def flops_per_rank(self) -> float:
        """Actual FLOPs one rank executes (the harness reports 2mnk)."""
        return 2.0 * self.m * self.n * self.k

    def as_tuple(self) -> Tuple[str, int, int, int]:
        return (self.primitive, self.m, self.n, self.k)


def layer_gemms(model: str, tp: int, tokens: int) -> List[LayerGemm]:
    spec = MODELS[model]
    if spec.heads % tp or spec.ffn % tp or tokens % tp:
        raise ValueError(f"{model}: heads/ffn/tokens must be divisible by tp={tp}")
    kv = max(spec.kv_heads, tp)  # kv heads are replicated when tp > kv_heads
    qkv = (spec.heads + 2 * kv) * spec.head_dim
    up = spec.ffn * (2 if spec.gated_mlp else 1)
    return [
        LayerGemm("qkv_proj", "tp_columnwise", tokens, qkv // tp, spec.hidden),
        LayerGemm("attn_out_proj", "tp_rowwise", tokens, spec.hidden, spec.heads * spec.head_dim),
        LayerGemm("mlp_up_proj", "tp_columnwise", tokens, up // tp, spec.hidden),
        LayerGemm("mlp_down_proj", "tp_rowwise", tokens, spec.hidden, spec.ffn),
    ]


def benchmark_configs(model: str, tp: int, tokens: int, impls: Dict, dtype: str = "bfloat16",
                      **bench_kw) -> List[Dict]:
    """One ``run_benchmark`` config per layer GEMM (primitive-specific implementations)."""
    out = []
    for g in layer_gemms(model, tp, tokens):
        b = {"primitive": g.primitive, "m": g.m, "n": g.n, "k": g.k, "dtype": dtype,
             "validate": True, "num_iterations": 20, "num_warmups": 5,
             "implementations": impls, **bench_kw}
        b.setdefault("output_csv", f"results/{model}_tp{tp}_{g.name}_{{timestamp}}.csv")
        out.append({"benchmark": b, "gemm": g.name})
    return out
