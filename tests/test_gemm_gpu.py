"""Numerics of the CDNA4 MFMA GEMM against a plain PyTorch fp32 reference (GPU only).

Covers every dtype path (bf16/f16/f32/fp8/MX-fp8/f64-generic), every tile config, ragged M/N,
the generic fallback (odd K), grouped-row A/C addressing used by the pipelines, and an
identity-A / asymmetric-B check that catches a transposed C write (cdna guide §3).
"""

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ref(a, w):
    return a.to(torch.float32) @ w.to(torch.float32).t()


def _rand(shape, dtype, gen):
    x = torch.rand(shape, generator=gen, device=DEV, dtype=torch.float32) * 2 - 1
    return x.to(dtype)


def _tol(dtype, k):
    low = dtype in (torch.bfloat16, torch.float16, torch.float8_e4m3fn)
    return (1e-3 if low else 1e-4) * k


@pytest.fixture(scope="module")
def gen():
    g = torch.Generator(device=DEV)
    g.manual_seed(1234)
    return g


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("tile", ["256x256", "256x128", "128x256", "128x128", "256x256w4",
                                  "256x128w4", "i256", "i128", "i256w4", "t8", "pt8", "t4", "pt4"])
def test_gemm_tiles(dtype, tile, gen):
    from ddlb_amd.ops.gemm import gemm

    M, N, K = 512, 384, 256
    a, w = _rand((M, K), dtype, gen), _rand((N, K), dtype, gen)
    out = gemm(a, w, tile=tile)
    torch.cuda.synchronize()
    assert out.dtype == dtype
    torch.testing.assert_close(out.float(), _ref(a, w), rtol=0, atol=_tol(dtype, K))


@pytest.mark.parametrize("shape", [(1000, 300, 128), (17, 1024, 512), (256, 4, 64), (1, 1, 64)])
def test_gemm_ragged_mn(shape, gen):
    from ddlb_amd.ops.gemm import gemm

    M, N, K = shape
    a, w = _rand((M, K), torch.bfloat16, gen), _rand((N, K), torch.bfloat16, gen)
    out = gemm(a, w)
    torch.cuda.synchronize()
    torch.testing.assert_close(out.float(), _ref(a, w), rtol=0, atol=_tol(torch.bfloat16, K))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32, torch.float64])
def test_gemm_generic_fallback(dtype, gen):
    from ddlb_amd.ops.gemm import gemm

    M, N, K = 130, 70, 100  # K*esize not a multiple of 128 -> generic kernel
    a, w = _rand((M, K), dtype, gen), _rand((N, K), dtype, gen)
    out = gemm(a, w)
    torch.cuda.synchronize()
    torch.testing.assert_close(out.double(), (a.double() @ w.double().t()), rtol=0,
                               atol=_tol(dtype, K))


def test_identity_asymmetric(gen):
    from ddlb_amd.ops.gemm import gemm

    M = N = K = 256
    a = torch.eye(M, device=DEV, dtype=torch.bfloat16)
    i = torch.arange(N, device=DEV).view(-1, 1).float()
    j = torch.arange(K, device=DEV).view(1, -1).float()
    w = ((i * 3 + j * 7) % 61 - 30).to(torch.bfloat16)  # asymmetric, exact in bf16
    out = gemm(a, w)
    torch.cuda.synchronize()
    assert torch.equal(out.float(), w.float().t())


@pytest.mark.parametrize("mode", ["auto", "mx"])
@pytest.mark.parametrize("odt", [torch.bfloat16, torch.float32])
def test_gemm_fp8(mode, odt, gen):
    from ddlb_amd.ops.gemm import gemm

    M, N, K = 512, 256, 512
    a = _rand((M, K), torch.float8_e4m3fn, gen)
    w = _rand((N, K), torch.float8_e4m3fn, gen)
    out = gemm(a, w, out_dtype=odt, mode=mode)
    torch.cuda.synchronize()
    torch.testing.assert_close(out.float(), _ref(a, w), rtol=0, atol=_tol(torch.float8_e4m3fn, K))


@pytest.mark.parametrize("tile", ["auto", "128x128", "256x256w4", "256x128w4", "i256", "i128",
                                  "i256w4", "t8", "pt8", "t4", "pt4"])
def test_fp8_integer_exact(gen, tile):
    """Small integers are exact in e4m3: both fp8 paths must match bit for bit."""
    from ddlb_amd.ops.gemm import gemm

    M, N, K = 512, 256, 512
    a = torch.randint(-3, 4, (M, K), device=DEV, generator=gen).float().to(torch.float8_e4m3fn)
    w = torch.randint(-3, 4, (N, K), device=DEV, generator=gen).float().to(torch.float8_e4m3fn)
    ref = _ref(a, w)
    for mode in ("auto", "mx"):
        out = gemm(a, w, out_dtype=torch.float32, mode=mode, tile=tile)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), mode


def test_grouped_rows(gen):
    """Pipeline addressing: A rows from strided blocks, C rows to strided blocks."""
    from ddlb_amd.ops.gemm import gemm

    d, blk, K, N = 4, 256, 256, 512
    A = _rand((d * 1024, K), torch.bfloat16, gen)     # d blocks of 1024 rows
    w = _rand((N, K), torch.bfloat16, gen)
    C = torch.zeros((d * 1024, N), dtype=torch.bfloat16, device=DEV)
    j = 2  # stage 2 of 4: rows j*blk..(j+1)*blk of every block
    gemm(A[j * blk:], w, C[j * blk:], M=d * blk, a_grp=blk, a_gstride=1024, c_grp=blk,
         c_gstride=1024)
    torch.cuda.synchronize()
    ref = _ref(A, w)
    for r in range(d):
        rows = slice(r * 1024 + j * blk, r * 1024 + (j + 1) * blk)
        torch.testing.assert_close(C[rows].float(), ref[rows], rtol=0, atol=0.3)
    untouched = torch.ones(d * 1024, dtype=torch.bool, device=DEV)
    for r in range(d):
        untouched[r * 1024 + j * blk:r * 1024 + (j + 1) * blk] = False
    assert torch.count_nonzero(C[untouched].float()) == 0


@pytest.mark.parametrize("tile", ["auto", "128x128", "256x256w4", "256x128w4", "i256", "i128",
                                  "i256w4", "t8", "pt8", "t4", "pt4"])
@pytest.mark.parametrize("shape", [(2048, 1024, 1024), (4096, 2048, 2048), (768, 512, 192)])
def test_repeat_race_screen(gen, tile, shape):
    """Same inputs, 20 launches: identical bits every time (LDS-DMA/barrier race screen)."""
    from ddlb_amd.ops.gemm import gemm

    M, N, K = shape
    a, w = _rand((M, K), torch.bfloat16, gen), _rand((N, K), torch.bfloat16, gen)
    first = gemm(a, w, tile=tile).clone()
    out = torch.empty_like(first)
    for _ in range(20):
        gemm(a, w, out, tile=tile)
        torch.cuda.synchronize()
        assert torch.equal(out, first)
    torch.testing.assert_close(first.float(), _ref(a, w), rtol=0, atol=_tol(torch.bfloat16, K))


def test_host_checks_reject_bad_shapes(gen):
    from ddlb_amd.ops.gemm import gemm

    a = _rand((64, 128), torch.bfloat16, gen)
    w = _rand((64, 96), torch.bfloat16, gen)
    with pytest.raises(ValueError):
        gemm(a, w)
    with pytest.raises(ValueError):
        gemm(a, _rand((64, 128), torch.bfloat16, gen), M=128)


@pytest.mark.parametrize("tile", ["pt8", "pt4"])
def test_persistent_many_tiles_grouped(gen, tile):
    """Persistent streaming kernel: more tiles than blocks, grouped C rows, repeat-identical."""
    from ddlb_amd.ops.gemm import gemm

    M, N, K = 8192, 1024, 512
    a, w = _rand((M, K), torch.bfloat16, gen), _rand((N, K), torch.bfloat16, gen)
    out = torch.zeros((2 * M, N), dtype=torch.bfloat16, device=DEV)
    gemm(a, w, out, tile=tile, c_grp=1024, c_gstride=2048)
    torch.cuda.synchronize()
    ref = _ref(a, w)
    for blk in range(M // 1024):
        torch.testing.assert_close(out[blk * 2048:blk * 2048 + 1024].float(),
                                   ref[blk * 1024:(blk + 1) * 1024], rtol=0, atol=_tol(torch.bfloat16, K))
        assert torch.count_nonzero(out[blk * 2048 + 1024:(blk + 1) * 2048]) == 0
    first = out.clone()
    for _ in range(10):
        gemm(a, w, out, tile=tile, c_grp=1024, c_gstride=2048)
    torch.cuda.synchronize()
    assert torch.equal(out, first)


@pytest.mark.parametrize("act", ["gelu", "relu", "silu"])
@pytest.mark.parametrize("tile", ["auto", "128x128", "i256", "t8", "pt8", "t4", "pt4"])
def test_fused_activation_epilogue(gen, act, tile):
    from ddlb_amd.ops.gemm import gemm
    from ddlb_amd.parallel.sim import apply_act

    M, N, K = 512, 512, 256
    a, w = _rand((M, K), torch.bfloat16, gen), _rand((N, K), torch.bfloat16, gen)
    out = gemm(a, w, tile=tile, act=act)
    torch.cuda.synchronize()
    code = {"gelu": 1, "relu": 2, "silu": 3}[act]
    torch.testing.assert_close(out.float(), apply_act(_ref(a, w), code), rtol=0.02, atol=0.05)


_ALL_DT = [(torch.bfloat16, torch.bfloat16), (torch.bfloat16, torch.float32),
            (torch.float16, torch.float16), (torch.float16, torch.float32),
            (torch.float32, torch.float32), (torch.float8_e4m3fn, torch.bfloat16),
            (torch.float8_e4m3fn, torch.float32)]


def test_retired_tiles_refused(gen):
    """The retired kernel families' codes (pp256 5, p256 8, p128 9, pi256 13, pi256w4 14, r256 15)
    are refused by the launcher: never silently rerouted to another kernel."""
    from ddlb_amd.ops import load

    a, w = _rand((512, 256), torch.bfloat16, gen), _rand((256, 256), torch.bfloat16, gen)
    out = torch.empty((512, 256), dtype=torch.bfloat16, device=DEV)
    for code in (5, 8, 9, 13, 14, 15, 20):
        with pytest.raises(RuntimeError):
            load().gemm(a.data_ptr(), w.data_ptr(), out.data_ptr(), 256, 256, 256, 512, 256, 256,
                        2, 2, code, 0, 0, 0, 0, 0, torch.cuda.current_stream().cuda_stream, 0)


@pytest.mark.parametrize("shape", [(256, 256, 128), (8192, 1024, 512), (32768, 1024, 256),
                                   (4096, 768, 1024)])
@pytest.mark.parametrize("dt", _ALL_DT, ids=lambda d: f"{str(d[0])[6:]}-{str(d[1])[6:]}")
def test_auto_every_dtype(dt, shape, gen):
    """auto tile (pt4 on whole grids, tiled kernels otherwise) for every input / output dtype:
    one tile, fewer tiles than CUs, several tiles per persistent block, N not a power of two;
    repeat-identical."""
    from ddlb_amd.ops.gemm import gemm

    din, dout = dt
    M, N, K = shape
    a, w = _rand((M, K), din, gen), _rand((N, K), din, gen)
    out = gemm(a, w, out_dtype=dout)
    torch.cuda.synchronize()
    assert out.dtype == dout
    torch.testing.assert_close(out.float(), _ref(a, w), rtol=0, atol=_tol(din, K))
    again = gemm(a, w, out_dtype=dout)
    torch.cuda.synchronize()
    assert torch.equal(out, again)


def test_no_vendor_mode(gen):
    """The native GEMM never dispatches to a vendor library: an unknown mode (the former
    hipBLASLt mode 3) is refused by the launcher, not silently routed anywhere."""
    from ddlb_amd.ops import load

    a, w = _rand((256, 256), torch.bfloat16, gen), _rand((256, 256), torch.bfloat16, gen)
    out = torch.empty((256, 256), dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError):
        load().gemm(a.data_ptr(), w.data_ptr(), out.data_ptr(), 256, 256, 256, 256, 256, 256,
                    2, 2, 0, 3, 0, 0, 0, 0, torch.cuda.current_stream().cuda_stream, 0)


@pytest.mark.parametrize("tile", ["t8", "pt8", "t4", "pt4"])
@pytest.mark.parametrize("dt", _ALL_DT, ids=lambda d: f"{str(d[0])[6:]}-{str(d[1])[6:]}")
@pytest.mark.parametrize("shape", [(256, 256, 64), (256, 256, 128), (8192, 1024, 512),
                                   (4096, 768, 1024), (2048, 2048, 3072), (65536, 1024, 128),
                                   (3328, 1536, 256)])  # grouped raster: 13 m-blocks, 6 n
def test_t8_kernel(dt, shape, gen, tile):
    """8-phase ping-pong kernel and its persistent form: one K-tile (the clamped prefetch path),
    two, odd K-tile counts, N not a power of two, several tiles per persistent block (C quadrant
    stores in flight across the next tile's staging); every input/output dtype; repeat-identical."""
    from ddlb_amd.ops.gemm import gemm

    din, dout = dt
    M, N, K = shape
    if K * din.itemsize % 128:
        pytest.skip("K row must be a whole number of 128-byte K-tiles")
    a, w = _rand((M, K), din, gen), _rand((N, K), din, gen)
    out = gemm(a, w, tile=tile, out_dtype=dout)
    torch.cuda.synchronize()
    assert out.dtype == dout
    torch.testing.assert_close(out.float(), _ref(a, w), rtol=0, atol=_tol(din, K))
    again = gemm(a, w, tile=tile, out_dtype=dout)
    torch.cuda.synchronize()
    assert torch.equal(out, again)


@pytest.mark.parametrize("tile", ["t8", "pt8", "t4", "pt4"])
def test_t8_grouped_rows_and_race_screen(gen, tile):
    """t8 with the pipelines' strided A and C row blocks, then 50 launches of a large square
    GEMM compared bit for bit (a new sync template: RAW/WAR screen over many runs)."""
    from ddlb_amd.ops.gemm import gemm

    d, blk, K, N = 4, 512, 256, 1024
    A = _rand((d * 2048, K), torch.bfloat16, gen)
    w = _rand((N, K), torch.bfloat16, gen)
    C = torch.zeros((d * 2048, N), dtype=torch.bfloat16, device=DEV)
    gemm(A[blk:], w, C[blk:], M=d * blk, a_grp=blk, a_gstride=2048, c_grp=blk, c_gstride=2048,
         tile=tile)
    torch.cuda.synchronize()
    ref = _ref(A, w)
    for r in range(d):
        rows = slice(r * 2048 + blk, r * 2048 + 2 * blk)
        torch.testing.assert_close(C[rows].float(), ref[rows], rtol=0, atol=_tol(torch.bfloat16, K))
    a, w = _rand((4096, 4096), torch.bfloat16, gen), _rand((4096, 4096), torch.bfloat16, gen)
    first = gemm(a, w, tile=tile).clone()
    out = torch.empty_like(first)
    for _ in range(50):
        gemm(a, w, out, tile=tile)
    torch.cuda.synchronize()
    assert torch.equal(out, first)
    torch.testing.assert_close(first.float(), _ref(a, w), rtol=0, atol=_tol(torch.bfloat16, 4096))


@pytest.mark.parametrize("tile", ["t8", "pt8", "t4", "pt4"])
@pytest.mark.parametrize("shape", [(256, 256, 128), (2048, 768, 1024), (65536, 1024, 256)])
def test_t8_mx_fp8(tile, shape, gen):
    """Block-scaled MX-fp8 on the 8-phase schedule (one 16x16x128 scaled MFMA per 128-byte
    K-row): integer data is exact, random data within the fp8 tolerance; repeat-identical."""
    from ddlb_amd.ops.gemm import gemm

    M, N, K = shape
    a = torch.randint(-3, 4, (M, K), device=DEV, generator=gen).float().to(torch.float8_e4m3fn)
    w = torch.randint(-3, 4, (N, K), device=DEV, generator=gen).float().to(torch.float8_e4m3fn)
    out = gemm(a, w, out_dtype=torch.float32, mode="mx", tile=tile)
    torch.cuda.synchronize()
    assert torch.equal(out, _ref(a, w))
    a, w = _rand((M, K), torch.float8_e4m3fn, gen), _rand((N, K), torch.float8_e4m3fn, gen)
    out = gemm(a, w, mode="mx", tile=tile)
    torch.cuda.synchronize()
    torch.testing.assert_close(out.float(), _ref(a, w), rtol=0, atol=_tol(torch.float8_e4m3fn, K))
    again = gemm(a, w, mode="mx", tile=tile)
    torch.cuda.synchronize()
    assert torch.equal(out, again)


def _tight_bound(ref, k):
    """max|err| <= 2^-7 max|ref| + k 2^-12: output rounding plus f32 accumulation fit far inside;
    one dropped 16-byte K chunk per tile (error sigma ~0.9, max ~5 at k = 8192) does not — the
    reference's atol = 1e-3 k (8.2 at k = 8192) would let that through."""
    return 2.0 ** -7 * float(ref.abs().max()) + k * 2.0 ** -12


@pytest.mark.parametrize("tile", ["auto", "pt4", "t4", "t8", "pt8", "i256", "256x256",
                                  "128x128"])
@pytest.mark.parametrize("dt", [(torch.bfloat16, "auto"), (torch.float16, "auto"),
                                (torch.float8_e4m3fn, "mx"), (torch.float8_e4m3fn, "auto")],
                         ids=lambda d: f"{str(d[0])[6:]}-{d[1]}")
def test_gemm_long_k_tight(dt, tile, gen):
    """Every fast kernel at K = 8192 (the long-K shapes of BASELINE configs #2-#4) against the
    tight bound, with 512 x 512 outputs (several tiles, both wave groups, every K-tile kind)."""
    from ddlb_amd.ops.gemm import gemm

    dtype, mode = dt
    M, N, K = 512, 512, 8192
    a, w = _rand((M, K), dtype, gen), _rand((N, K), dtype, gen)
    out = gemm(a, w, tile=tile, mode=mode)
    torch.cuda.synchronize()
    ref = _ref(a, w)
    err = float((out.float() - ref).abs().max())
    assert err <= _tight_bound(ref, K), (err, _tight_bound(ref, K))


@pytest.mark.parametrize("dt", [(torch.bfloat16, torch.bfloat16, "auto"),
                                (torch.bfloat16, torch.float32, "auto"),
                                (torch.float8_e4m3fn, torch.bfloat16, "mx")],
                         ids=lambda d: f"{str(d[0])[6:]}-{str(d[1])[6:]}-{d[2]}")
@pytest.mark.parametrize("kt", [2, 3, 4, 5, 6, 12])
def test_pt4_k_tile_counts(dt, kt, gen):
    """pt4's tile body is unrolled by LDS-buffer parity (an even number of 128-byte K-tiles; odd
    counts go to t4) and its write-through form runs the DEFER schedule, whose K-tile kinds
    (first of the kernel, first after a tile, last, deferred A1 x B1) all meet within 2 - 12
    K-tiles and 8 tiles per persistent block; repeat-identical."""
    from ddlb_amd.ops.gemm import gemm

    din, dout, mode = dt
    K = kt * 128 // din.itemsize
    M, N = 2048 * 8, 256 * 8  # 512 tiles: two per persistent block
    a, w = _rand((M, K), din, gen), _rand((N, K), din, gen)
    out = gemm(a, w, tile="pt4", out_dtype=dout, mode=mode)
    torch.cuda.synchronize()
    ref = _ref(a, w)
    err = float((out.float() - ref).abs().max())
    assert err <= _tight_bound(ref, K), (err, K)
    again = gemm(a, w, tile="pt4", out_dtype=dout, mode=mode)
    torch.cuda.synchronize()
    assert torch.equal(out, again)


def test_pt4_flagship_race_screen(gen):
    """The flagship shape on pt4 (DEFER schedule, 4 tiles per block) 30 times, bit for bit: a
    new sync structure is screened over many runs (cdna_hip_programming.md §5, 8-phase notes)."""
    from ddlb_amd.ops.gemm import gemm

    a, w = _rand((65536, 1024), torch.bfloat16, gen), _rand((1024, 1024), torch.bfloat16, gen)
    first = gemm(a, w, tile="pt4").clone()
    out = torch.empty_like(first)
    for _ in range(30):
        gemm(a, w, out, tile="pt4")
        torch.cuda.synchronize()
        assert torch.equal(out, first)
    ref = _ref(a, w)
    assert float((first.float() - ref).abs().max()) <= _tight_bound(ref, 1024)


@pytest.mark.parametrize("dt", [(torch.bfloat16, torch.bfloat16, "auto"),
                                (torch.bfloat16, torch.float32, "auto"),
                                (torch.float8_e4m3fn, torch.bfloat16, "mx")],
                         ids=lambda d: f"{str(d[0])[6:]}-{str(d[1])[6:]}-{d[2]}")
@pytest.mark.parametrize("grp,cgrp", [(256, 0), (512, 512), (1024, 256)])
def test_pt4_grouped_a_rows(dt, grp, cgrp, gen):
    """pt4 reading A through grouped rows (groups of a multiple of 256 rows: one panel base per
    tile, the APAN instantiation) — the IPC / rowwise pipelines' stage GEMMs — with plain or
    grouped C, against the fp32 reference with the tight bound, repeat-identical 10x."""
    from ddlb_amd.ops.gemm import gemm

    din, dout, mode = dt
    d, K, N, stride = 8, 1024, 1024, 4096
    M = d * grp
    A = _rand((d * stride, K), din, gen)
    w = _rand((N, K), din, gen)
    C = torch.zeros((2 * M if cgrp else M, N), dtype=dout, device=DEV)
    kw = dict(M=M, a_grp=grp, a_gstride=stride, tile="pt4", out_dtype=dout, mode=mode)
    if cgrp:
        kw.update(c_grp=cgrp, c_gstride=2 * cgrp)
    gemm(A, w, C, **kw)
    torch.cuda.synchronize()
    idx = torch.cat([torch.arange(r * stride, r * stride + grp) for r in range(d)]).to(DEV)
    ref = _ref(A[idx], w)
    if cgrp:
        cidx = torch.cat([torch.arange(g * 2 * cgrp, g * 2 * cgrp + cgrp)
                          for g in range(M // cgrp)]).to(DEV)
        got = C[cidx]
    else:
        got = C
    err = float((got.float() - ref).abs().max())
    assert err <= _tight_bound(ref, K), err
    first = C.clone()
    for _ in range(10):
        gemm(A, w, C, **kw)
    torch.cuda.synchronize()
    assert torch.equal(C, first)


@pytest.mark.parametrize("ksplit", [0, 2, 4])
@pytest.mark.parametrize("dt", [(torch.bfloat16, "auto"), (torch.float16, "auto"),
                                (torch.float8_e4m3fn, "mx"), (torch.float8_e4m3fn, "auto")],
                         ids=lambda d: f"{str(d[0])[6:]}-{d[1]}")
def test_gemm_ksplit(dt, ksplit, gen):
    """K-split through ops.gemm (0 = the automatic rule, 4 slices for 2048 x 1024 x 8192's 32
    tiles; 2 / 4 explicit): one pt4 launch over (slice, tile) pairs + one reduce kernel, the
    tight bound at K = 8192 and repeat-identical."""
    from ddlb_amd.ops.gemm import gemm, split_k_factor

    dtype, mode = dt
    M, N, K = 2048, 1024, 8192
    assert split_k_factor(M, N, K, torch.tensor([], dtype=dtype).element_size()) == 4
    a, w = _rand((M, K), dtype, gen), _rand((N, K), dtype, gen)
    odt = torch.bfloat16 if dtype == torch.float8_e4m3fn else dtype
    out = torch.full((M, N), float("nan"), dtype=odt, device=DEV)
    gemm(a, w, out, mode=mode, ksplit=ksplit)
    torch.cuda.synchronize()
    ref = _ref(a, w)
    err = float((out.float() - ref).abs().max())
    assert err <= _tight_bound(ref, K), err
    first = out.clone()
    for _ in range(5):
        gemm(a, w, out, mode=mode, ksplit=ksplit)
    torch.cuda.synchronize()
    assert torch.equal(out, first)
