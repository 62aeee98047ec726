"""Worker for tests/test_gemm_gpu.py::test_pt4_schedule_knobs: the pt4 launcher reads its A/B
knobs (DDLB_PT4_ONE, DDLB_PT4_HALF_LINES, DDLB_PT4_C_NT) once per process, so each knob runs in a
process of its own. Checks the ungated write-through pt4 -- the instantiation the knobs switch --
against the fp32 product with the tight bound on a few shapes and dtypes, and that a repeat is
bit-identical. Prints one JSON line: {"knob": ..., "cases": n, "worst": max err / bound}.
"""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from ddlb_amd.ops.gemm import gemm

    knob = os.environ.get("DDLB_TEST_KNOB", "")
    gen = torch.Generator(device="cuda")
    gen.manual_seed(7)
    cases = [  # (M, N, K, in dtype, out dtype, mode): whole 256x256 tiles, nk >= 4
        (8192, 1024, 1024, torch.bfloat16, torch.bfloat16, "auto"),
        (4096, 2048, 4096, torch.bfloat16, torch.bfloat16, "auto"),
        (4096, 1024, 2048, torch.float16, torch.float16, "auto"),
        (8192, 1024, 1024, torch.float8_e4m3fn, torch.bfloat16, "mx"),
        (4096, 512, 4096, torch.float8_e4m3fn, torch.bfloat16, "auto"),
    ]
    worst = 0.0
    for M, N, K, dt, odt, mode in cases:
        a = (torch.rand((M, K), generator=gen, device="cuda") * 2 - 1).to(dt)
        w = (torch.rand((N, K), generator=gen, device="cuda") * 2 - 1).to(dt)
        out = torch.full((M, N), float("nan"), dtype=odt, device="cuda")
        gemm(a, w, out, tile="pt4", mode=mode, ksplit=1)
        torch.cuda.synchronize()
        ref = a.float() @ w.float().t()
        bound = 2.0 ** -7 * float(ref.abs().max()) + K * 2.0 ** -12
        err = float(torch.nan_to_num((out.float() - ref).abs(), nan=float("inf")).max())
        worst = max(worst, err / bound)
        again = torch.empty_like(out)
        gemm(a, w, again, tile="pt4", mode=mode, ksplit=1)
        torch.cuda.synchronize()
        if not torch.equal(again, out):
            worst = float("inf")
    print(json.dumps({"knob": knob, "cases": len(cases), "worst": worst}), flush=True)


if __name__ == "__main__":
    main()
