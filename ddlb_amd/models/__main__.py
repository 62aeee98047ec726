"""Benchmark the TP GEMMs of one transformer layer of a real model.

    python -m ddlb_amd.models --model llama3-70b --tp 8 --tokens 8192 --list
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m ddlb_amd.models \
        --model llama3-70b --tokens 8192 --impl "native;algorithm=coll_pipeline;s=4" \
        --impl "pytorch;empty_cache=false"
"""

from __future__ import annotations

import argparse

from ddlb_amd.cli.config import parse_impl_spec
from ddlb_amd.envs import get_rank, get_world_size
from ddlb_amd.models.shapes import MODELS, benchmark_configs, layer_gemms


def main(argv=None) -> None:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--model", required=True, choices=sorted(MODELS))
    p.add_argument("--tp", type=int, default=0, help="default: the world size")
    p.add_argument("--tokens", type=int, default=8192)
    p.add_argument("--dtype", default="bfloat16")
    p.add_argument("--impl", action="append", default=None)
    p.add_argument("--num-iterations", type=int, default=20)
    p.add_argument("--list", action="store_true", help="print the GEMMs and exit")
    a = p.parse_args(argv)
    tp = a.tp or get_world_size()
    gemms = layer_gemms(a.model, tp, a.tokens)
    if a.list or get_rank() == 0:
        for g in gemms:
            print(f"{a.model} tp={tp} {g.name:14s} {g.primitive:14s} m={g.m} n={g.n} k={g.k}")
    if a.list:
        return
    impls = {}
    for spec in a.impl or ["native;algorithm=coll_pipeline;s=4", "pytorch;empty_cache=false"]:
        name, opts = parse_impl_spec(spec)
        impls.setdefault(name, []).append(opts)
    from ddlb_amd.cli.benchmark import run_benchmark

    for cfg in benchmark_configs(a.model, tp, a.tokens, impls, dtype=a.dtype,
                                 num_iterations=a.num_iterations):
        if get_rank() == 0:
            print(f"\n=== {cfg['gemm']} ===")
        run_benchmark({"benchmark": cfg["benchmark"]})


if __name__ == "__main__":
    main()
