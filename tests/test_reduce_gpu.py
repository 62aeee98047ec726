"""The d-way reduce kernel of the native reduce-scatter (`csrc/runtime/kernels.hip`): every
source count (the fixed-count unrolled kernels 2..8 and the runtime-count kernel beyond), every
dtype, ragged tails; compared with an fp32 PyTorch sum in the same source order."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}


@pytest.mark.parametrize("dtype", list(DT))
@pytest.mark.parametrize("nsrc", [1, 2, 3, 4, 5, 7, 8, 9, 16])
@pytest.mark.parametrize("count", [8, 1000, 1 << 20])
def test_reduce_sum(dtype, nsrc, count):
    from ddlb_amd.ops import load

    C = load()
    gen = torch.Generator(device="cuda").manual_seed(nsrc * 131 + count)
    # 16-byte aligned sources: one slab, rows padded to a multiple of 8 elements
    pad = (count + 7) // 8 * 8
    slab = torch.rand((nsrc, pad), generator=gen, device="cuda", dtype=torch.float32)
    slab = (2 * slab - 1).to(dtype)
    out = torch.full((pad,), float("nan"), device="cuda", dtype=dtype)
    s = torch.cuda.current_stream().cuda_stream
    C.reduce_sum(out.data_ptr(), [slab[i].data_ptr() for i in range(nsrc)], count, DT[dtype], s)
    torch.cuda.synchronize()
    ref = slab[0, :count].float()
    for i in range(1, nsrc):
        ref = ref + slab[i, :count].float()
    tol = 1e-6 if dtype == torch.float32 else 1e-2 * nsrc
    torch.testing.assert_close(out[:count].float(), ref.to(dtype).float(), rtol=0, atol=tol)
    if pad > count:
        assert torch.isnan(out[count:].float()).all()  # nothing written past count


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("nsrc", [1, 2, 4, 8, 9])
@pytest.mark.parametrize("count", [8, 1003, (1 << 20) + 5])
def test_reduce_sum_f32_sources(dtype, nsrc, count):
    """f32 sources into a 16-bit destination (the K-split GEMM's partials, rounded once): equal
    to the fp32 sum in source order, rounded to the destination dtype."""
    from ddlb_amd.ops import load

    C = load()
    gen = torch.Generator(device="cuda").manual_seed(nsrc * 7 + count)
    pad = (count + 7) // 8 * 8
    slab = 2 * torch.rand((nsrc, pad), generator=gen, device="cuda", dtype=torch.float32) - 1
    out = torch.full((pad,), float("nan"), device="cuda", dtype=dtype)
    s = torch.cuda.current_stream().cuda_stream
    C.reduce_sum(out.data_ptr(), [slab[i].data_ptr() for i in range(nsrc)], count, DT[dtype], s,
                 DT[torch.float32])
    torch.cuda.synchronize()
    ref = slab[0, :count].clone()
    for i in range(1, nsrc):
        ref = ref + slab[i, :count]
    assert torch.equal(out[:count], ref.to(dtype))
    if pad > count:
        assert torch.isnan(out[count:].float()).all()
    with pytest.raises(RuntimeError):  # f32 sources only, 16-bit destinations only
        C.reduce_sum(out.data_ptr(), [slab[0].data_ptr()], count, DT[dtype], s, DT[dtype] ^ 3)
