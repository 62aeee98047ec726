"""Python front-end of the CDNA4 MFMA GEMM (``csrc/gemm/gemm_mfma.hip``).

``gemm(a, w)`` computes ``a @ w.T`` for ``a: [M, K]`` and ``w: [N, K]`` (the weight kept
K-contiguous, like ``te.Linear``'s ``[out, in]``), with optional grouped-row addressing of A and C:
logical row ``i`` lives at physical row ``base + (i // grp) * gstride + i % grp``.

Every shape / dtype / device / alignment / bounds check happens here, on the host, before the
kernel launches (a bad launch can fault every GPU of the node).

dtypes: bf16 -> bf16|f32, f16 -> f16|f32, f32 -> f32 (exact f32 MFMA), float8_e4m3fn -> bf16|f16|f32
(``mx=True``: block-scaled MX-fp8 MFMA at 2x the bf16 rate, unit scales), f64 (generic kernel).
"""

from __future__ import annotations

from typing import Optional

from ddlb_amd.ops import load

DT_F32, DT_F16, DT_BF16, DT_FP8, DT_F64, DT_U8 = 0, 1, 2, 3, 4, 5
# (codes 5, 8, 9, 13-15 belonged to the pp256 / p256 / p128 / pi256 / pi256w4 / r256 families,
# retired in round 4: no auto path reached them and pt4 superseded them on every shape measured)
TILES = {"auto": 0, "256x256": 1, "256x128": 2, "128x256": 3, "128x128": 4, "256x256w4": 6,
         "256x128w4": 7, "i256": 10, "i128": 11, "i256w4": 12,
         "t8": 16, "pt8": 17, "t4": 18, "pt4": 19}
MODES = {"auto": 0, "generic": 1, "mx": 2}
ACTS = {"none": 0, "gelu": 1, "relu": 2, "silu": 3}

SUPPORTED_IN = ("float32", "float16", "bfloat16", "float8_e4m3fn", "float64")


def dtype_code(dt) -> int:
    import torch

    table = {torch.float32: DT_F32, torch.float16: DT_F16, torch.bfloat16: DT_BF16,
             torch.float8_e4m3fn: DT_FP8, torch.float64: DT_F64, torch.uint8: DT_U8}
    if dt not in table:
        raise TypeError(f"dtype {dt} is not supported by the native GEMM")
    return table[dt]


def check_supported(dtype_name: str) -> None:
    if dtype_name not in SUPPORTED_IN:
        raise TypeError(f"native GEMM supports {SUPPORTED_IN}, not {dtype_name}")


def default_out_dtype(in_dtype):
    import torch

    return torch.bfloat16 if in_dtype == torch.float8_e4m3fn else in_dtype


def _check_operands(a, w, out, M, a_rows_phys):
    import torch

    if a.device.type != "cuda" or w.device.type != "cuda" or out.device.type != "cuda":
        raise ValueError("native GEMM operands must be ROCm device tensors")
    if not (a.device == w.device == out.device):
        raise ValueError("operands on different devices")
    if a.dim() != 2 or w.dim() != 2 or out.dim() != 2:
        raise ValueError("native GEMM expects 2-D operands")
    if a.stride(1) != 1 or w.stride(1) != 1 or out.stride(1) != 1:
        raise ValueError("operands must be row-major with unit inner stride")
    if a.dtype != w.dtype:
        raise TypeError(f"A dtype {a.dtype} != W dtype {w.dtype}")
    if a.shape[1] != w.shape[1]:
        raise ValueError(f"K mismatch: A {tuple(a.shape)} vs W {tuple(w.shape)}")
    if out.shape[1] < w.shape[0]:
        raise ValueError(f"output has {out.shape[1]} columns < N={w.shape[0]}")
    if a_rows_phys > a.shape[0]:
        raise ValueError(f"A row mapping reaches row {a_rows_phys - 1} >= {a.shape[0]}")
    if a.dtype == torch.float8_e4m3fn and out.dtype not in (torch.bfloat16, torch.float16,
                                                             torch.float32):
        raise TypeError("fp8 GEMM output must be bf16, f16 or f32")


def _phys_rows(M: int, grp: int, gstride: int, base_rows: int = 0) -> int:
    """One past the largest physical row the mapping touches."""
    if M == 0:
        return 0
    if grp <= 0:
        return M
    last = M - 1
    return (last // grp) * gstride + (last % grp) + 1


def device_cus() -> int:
    """CUs of the current device (256 on a whole MI355X; fewer in a compute partition), 256 when
    no GPU is visible (plans built on the CPU)."""
    import torch

    if not torch.cuda.is_available():
        return 256
    return int(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count)


def split_k_factor(M: int, N: int, K: int, esz: int, ncu: int = 0) -> int:
    """K-slices for a GEMM whose 256x256 grid covers at most half the CUs and whose K is long
    (e.g. 8192 x 1024 x 8192: 128 tiles): ``S`` slices run as (slice, tile) pairs of ONE pt4
    launch (``GemmArgs::ksplit``), their partials summed by the reduce kernel. Each slice
    keeps >= 16 K-tiles (the fixed per-tile cost stays small, profiles/r04/r4_15_*); measured
    on the config #2 shape: 0.1009 ms vs 0.1338 unsplit (profiles/r04/r4_22_*). 1 = no split."""
    if M % 256 or N % 256 or M <= 0 or N <= 0:
        return 1
    ncu = ncu or device_cus()
    tiles = (M // 256) * (N // 256)
    nk = K * esz // 128
    if K * esz % 128:
        return 1
    for S in (4, 2):
        if tiles * S <= ncu and nk % (2 * S) == 0 and nk // S >= 16:
            return S
    return 1


def gemm(a, w, out=None, *, out_dtype=None, tile: str = "auto", mode: str = "auto",
         M: Optional[int] = None, a_grp: int = 0, a_gstride: int = 0, c_grp: int = 0,
         c_gstride: int = 0, stream=None, act: str = "none", ksplit: int = 0):
    """``out[:M] = act(a[:M] @ w.T)`` on the current HIP stream (grouped-row addressing and a
    fused epilogue activation — none / gelu (tanh) / relu / silu — optional). ``ksplit``: 0 =
    auto (:func:`split_k_factor` for plain-row auto-tile GEMMs with no activation and a dense
    output), 1 = never, S > 1 = S slices. A pt4 split runs one launch over (slice, tile) pairs
    into f32 partials, summed in slice order and rounded once by the reduce kernel (0.1122 ms on
    8192 x 1024 x 8192 bf16, ``profiles/r05/r5_14_*``)."""
    import torch

    C = load()
    if out is None:
        rows = M if M is not None else a.shape[0]
        out = torch.empty((rows, w.shape[0]), dtype=out_dtype or default_out_dtype(a.dtype),
                          device=a.device)
    M = a.shape[0] if M is None else int(M)
    N, K = w.shape
    a_need = _phys_rows(M, a_grp, a_gstride)
    c_need = _phys_rows(M, c_grp, c_gstride)
    _check_operands(a, w, out, M, a_need)
    if c_need > out.shape[0]:
        raise ValueError(f"C row mapping reaches row {c_need - 1} >= {out.shape[0]}")
    if a_grp and (a_grp < 0 or a_gstride < a_grp):
        raise ValueError("a_gstride must be >= a_grp")
    if c_grp and (c_grp < 0 or c_gstride < c_grp):
        raise ValueError("c_gstride must be >= c_grp")
    if M >= 2 ** 31 or N >= 2 ** 31 or K >= 2 ** 31:
        raise ValueError("dimensions must fit in 32 bits")
    s = stream if stream is not None else torch.cuda.current_stream(a.device).cuda_stream
    plain = (a_grp in (0, M) and c_grp in (0, M) and ACTS[act] == 0 and out.stride(0) == N
             and mode != "generic" and a.dtype != torch.float64)
    S = int(ksplit)
    if S == 0:
        S = split_k_factor(M, N, K, a.element_size()) if plain and tile == "auto" else 1
    if S > 1:
        if not plain or K % S or M % 256 or N % 256:
            raise ValueError("ksplit needs plain rows, no activation, a dense output, whole "
                             "256x256 tiles and S | K")
        if tile not in ("auto", "pt4"):
            # another kernel runs the slices one after another into output-dtype partials,
            # summed (f32) by a reduce kernel
            part = torch.empty((S, M, N), dtype=out.dtype, device=a.device)
            C.gemm(a.data_ptr(), w.data_ptr(), part.data_ptr(), a.stride(0), w.stride(0), N, M,
                   N, K // S, dtype_code(a.dtype), dtype_code(out.dtype), TILES[tile],
                   MODES[mode], 0, 0, 0, 0, s, 0, S)
            C.reduce_sum(out.data_ptr(), [part[j].data_ptr() for j in range(S)], M * N,
                         dtype_code(out.dtype), s)
            if stream is not None:
                part.record_stream(torch.cuda.ExternalStream(s))
            return out
        # every (slice, tile) pair in one launch into f32 partials, summed in slice order and
        # rounded once by the reduce kernel (an unsplit GEMM's rounding)
        ws = torch.empty((S, M, N), dtype=torch.float32, device=a.device)
        C.gemm(a.data_ptr(), w.data_ptr(), ws.data_ptr(), a.stride(0), w.stride(0), N, M, N,
               K // S, dtype_code(a.dtype), DT_F32, TILES["pt4"], MODES[mode], 0, 0, 0, 0, s, 0, S)
        if out.dtype == torch.float32:
            C.reduce_sum(out.data_ptr(), [ws[j].data_ptr() for j in range(S)], M * N, DT_F32, s)
        else:
            C.reduce_sum(out.data_ptr(), [ws[j].data_ptr() for j in range(S)], M * N,
                         dtype_code(out.dtype), s, DT_F32)
        if stream is not None:  # the workspace stays allocated until that stream reaches it
            ws.record_stream(torch.cuda.ExternalStream(s))
        return out
    C.gemm(a.data_ptr(), w.data_ptr(), out.data_ptr(), a.stride(0), w.stride(0), out.stride(0),
           M, N, K, dtype_code(a.dtype), dtype_code(out.dtype), TILES[tile], MODES[mode],
           a_grp, a_gstride, c_grp, c_gstride, s, ACTS[act])
    return out


def fast_path_ok(a, w, out) -> bool:
    C = load()
    return bool(C.gemm_fast_path_ok(a.data_ptr(), w.data_ptr(), out.data_ptr(), a.stride(0),
                                    w.stride(0), out.stride(0), a.shape[0], w.shape[0],
                                    a.shape[1], dtype_code(a.dtype), dtype_code(out.dtype)))
