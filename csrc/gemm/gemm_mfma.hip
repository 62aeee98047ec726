// CDNA4 (gfx950) MFMA GEMM:  C[M,N] = A[M,K] * Bt[N,K]^T  ("TN": both operands K-contiguous).
//
// Replaces the cuBLAS GEMM the reference reaches through torch.matmul
// (ddlb/primitives/TPColumnwise/pytorch.py:97, TPRowwise/pytorch.py:82, compute_only.py:40).
//
// Design (see /opt/skills/guides/cdna_hip_programming.md §5):
//  * Operands staged global->LDS with LDS-DMA (`global_load_lds_dwordx4`, 16 B/lane, 1 KiB per
//    wave-instruction), double-buffered, one barrier per K-tile (the "minimum 2-phase" schedule).
//  * Every K-tile row is 128 bytes (BK = 64 for 16-bit types, 128 for fp8, 32 for fp32), so one
//    LDS layout serves every dtype. 16-byte chunks are XOR-swizzled with (row>>1)&7; because the
//    LDS-DMA destination is lane-linear, the swizzle is applied to the per-lane SOURCE address and
//    undone on the ds_read_b128 (rule 21). Conflict-free for the 16x16 fragment reads.
//  * MFMA 16x16x32 (bf16/f16), 2x 16x16x32 fp8 per 16 B, 4x 16x16x4 f32 per 16 B, or the
//    block-scaled 16x16x128 f8f6f4 (MX-fp8, unit scales) that runs at 2x the bf16 rate.
//    Any k-permutation that is identical for A and B leaves the dot product unchanged, which is
//    what lets one 16-byte ds_read feed every instruction shape.
//  * Operands are swapped in the MFMA (D = Bt_frag x A_frag) so each lane ends with 4 consecutive
//    COLUMNS of one C row: the epilogue is one 8-byte (bf16) / 16-byte (f32) store per fragment.
//  * Grouped-row addressing for A and C: logical row i lives at physical row
//        base + (i / grp) * gstride + (i % grp)
//    so pipeline stages read strided row blocks of A and write straight to their final rows of C
//    (no permutation copy).
//  * Bijective XCD-aware block remap (8 XCDs, private L2s): blocks that share an A panel land on
//    the same XCD.
//  * Optional arrival flags: a tile whose A rows belong to shard s spins (bounded) until
//    flags[s] >= epoch before loading A, so one persistent-size GEMM launch can consume shards as
//    the copy engines deliver them (p2p pipeline).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>


#include "gemm.h"
#include "gemm_entry.h"

namespace ddlb {

int tile_rows(int tile) {
  return (tile == TILE_128x128 || tile == TILE_128x256 || tile == TILE_I128) ? 128 : 256;
}
int tile_cols(int tile) {
  return (tile == TILE_256x128 || tile == TILE_128x128 || tile == TILE_256x128_W4 ||
          tile == TILE_I128) ? 128 : 256;
}

bool gemm_fast_path_ok(const GemmArgs& p, int din, int dout) {
  const int esz = dtype_size(din);
  if (din == DT_F64 || (din == DT_FP8 && dout == DT_FP8)) return false;
  if (p.M <= 0 || p.N <= 0 || p.K <= 0) return false;
  if ((int64_t)p.K * esz % 128 != 0) return false;
  if (p.lda * esz % 16 || p.ldb * esz % 16) return false;
  if (((uintptr_t)p.a | (uintptr_t)p.b) & 15) return false;
  if ((p.ldc * dtype_size(dout)) % 8 || ((uintptr_t)p.c & 7)) return false;
  if (p.a_grp <= 0 || p.c_grp <= 0) return false;
  return true;
}

int choose_tile(int64_t M, int64_t N, int64_t K, int din) {
  // Measured on MI355X: among the ping-pong kernels, pt4 (t4 made persistent) leads t4 / t8 / pt8
  // on every shape and dtype measured once the C stores are non-temporal
  // (profiles/r01/s2/s2_41_tune_nt.txt: bf16 flagship 108.9 vs t4 121.1 us, 16384x8192x1024
  // 231.7 vs 251.9, 8192^3 695.7 vs 703.4; s2_44_fp8_tiles.txt: MX-fp8 flagship 63.6 vs pt8
  // 67.4 us, 8192^3 363 vs t8 380) whenever the grid covers most of the CUs; it falls back to t4
  // where it does not apply (a single K-tile, an odd K-tile count, activations). Long K with
  // fewer whole tiles prefers the 128-byte-row interleaved kernel; fewer tiles than CUs want
  // 128x128 blocks. (The LDS-ring, 256x256 ping-pong and persistent streaming families this
  // table once chose between were retired in round 4: pt4 had superseded them on every shape.)
  auto tiles = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  (void)K;
  (void)din;
  // (down to half the CUs' worth of 256x256 tiles: at 128 tiles pt4 still beats the 128x128
  // kernel, 8192x1024x1024 bf16 22.5 vs 23.0 us, MX-fp8 14.8 vs 16.4, profiles/r04/r4_24_*)
  const bool whole = M % 256 == 0 && N % 256 == 0 && tiles(256, 256) >= 128;
  if (whole) return TILE_PT4;
  if (tiles(256, 256) >= 384) return TILE_I256;
  if (tiles(256, 128) >= 384) return TILE_256x128;
  if (tiles(128, 256) >= 384) return TILE_128x256;
  return TILE_128x128;
}

hipError_t gemm_launch(const GemmArgs& p_in, int din, int dout, int tile, int mode,
                       hipStream_t s) {
  GemmArgs p = p_in;
  if (p.a_grp <= 0) { p.a_grp = p.M > 0 ? p.M : 1; p.a_gstride = p.a_grp; }
  if (p.c_grp <= 0) { p.c_grp = p.M > 0 ? p.M : 1; p.c_gstride = p.c_grp; }
  switch (tile) {  // known codes only (the retired families' codes are refused, not rerouted)
    case TILE_AUTO: case TILE_256x256: case TILE_256x128: case TILE_128x256: case TILE_128x128:
    case TILE_256x256_W4: case TILE_256x128_W4: case TILE_I256: case TILE_I128: case TILE_I256W4:
    case TILE_T8: case TILE_PT8: case TILE_T4: case TILE_PT4: break;
    default: return hipErrorInvalidValue;
  }
  if (p.M == 0 || p.N == 0) return hipSuccess;
  if (p.ksplit > 1) {
    // K-split: slice j of K columns -> partial j at c + j * M * ldc (the caller sums them). pt4
    // runs every (slice, tile) pair in one launch; any other kernel runs the slices one by one.
    if (p.flags != nullptr || p.a_table != nullptr || p.c_table != nullptr || p.ag_ctas > 0 ||
        p.ag_mode != 0 || p.act != ACT_NONE || p.a_grp != p.M || p.c_grp != p.M || p.ksplit > 64)
      return hipErrorNotSupported;
    if (tile == TILE_AUTO || tile == TILE_PT4) {
      GemmArgs q = p;
      q.tile_order = 0;
      const bool fast = mode != GEMM_MODE_GENERIC && gemm_fast_path_ok(q, din, dout);
      hipError_t e = hipErrorNotSupported;
      if (fast && din == DT_FP8 && mode == GEMM_MODE_MX) e = launch_fast_mx(q, dout, TILE_PT4, s);
      else if (fast) e = launch_fast(q, din, dout, TILE_PT4, s);
      if (e != hipErrorNotSupported && e != hipErrorInvalidValue) return e;
    }
    const int esz = dtype_size(din), osz = dtype_size(dout);
    for (int j = 0; j < p.ksplit; ++j) {
      GemmArgs q = p;
      q.ksplit = 1;
      q.a = (const char*)p.a + (int64_t)j * p.K * esz;
      q.b = (const char*)p.b + (int64_t)j * p.K * esz;
      q.c = (char*)p.c + (int64_t)j * p.M * p.ldc * osz;
      const hipError_t e = gemm_launch(q, din, dout, tile == TILE_PT4 ? TILE_AUTO : tile, mode, s);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  if (p.a_table != nullptr) {
    // A through a row-block address table (direct access to the peers' shards, or the blocks of
    // a stage-major gather buffer): the ping-pong kernels (pt4 / t4 / t8 / pt8, whole 256-row
    // blocks; pt4 takes one panel base per tile) and the tiled kernels read A through it.
    // Arrival flags then index LOGICAL rows.
    if (p.shard_rows <= 0) return hipErrorInvalidValue;
    const bool whole = p.M % 256 == 0 && p.N % 256 == 0 && p.shard_rows % 256 == 0;
    if (tile == TILE_AUTO) {
      tile = choose_tile(p.M, p.N, p.K, din);
      if (tile != TILE_PT4 && tile != TILE_PT8 && tile != TILE_T4) tile = TILE_T8;
    }
    const bool ping = tile == TILE_T8 || tile == TILE_PT8 || tile == TILE_T4 || tile == TILE_PT4;
    if (ping && !whole) tile = TILE_128x128;
    // the tiled MX kernel addresses plain rows: block-scaled MFMAs on whole blocks only
    if (mode == GEMM_MODE_MX && !(ping && whole)) mode = GEMM_MODE_AUTO;
    if (p.flags != nullptr && !(ping && whole)) return hipErrorNotSupported;
    if (mode == GEMM_MODE_GENERIC || !gemm_fast_path_ok(p, din, dout)) return hipErrorNotSupported;
  }
  if (p.c_table != nullptr) {
    // direct-store C: every fast kernel addresses C rows through c_row(); the generic kernel
    // cannot, and an interleaved shard order needs whole tiles per shard
    if (p.c_shard_rows <= 0 || p.c_grp != p.M || mode == GEMM_MODE_GENERIC ||
        p.flags != nullptr || p.ag_ctas > 0 || !gemm_fast_path_ok(p, din, dout))
      return hipErrorNotSupported;
  }
  if (p.tile_order == 2 && (p.nshards <= 0 || p.M % p.nshards != 0))
    return hipErrorInvalidValue;
  if (p.ag_ctas > 0) {
    // in-kernel all-gather: only the gated persistent pt4 kernel carries the copy workgroups;
    // anything else would skip the copies, so refuse rather than fall back
    const int esz = dtype_size(din);
    if (p.flags == nullptr || p.a_table != nullptr || mode == GEMM_MODE_GENERIC ||
        !gemm_fast_path_ok(p, din, dout) || p.M % 256 || p.N % 256 || p.a_grp != p.M ||
        (int64_t)p.K * esz / 128 < 2 || ((int64_t)p.K * esz / 128) % 2 != 0 || p.act != ACT_NONE ||
        p.lda * esz > (1 << 22) || p.ldb * esz > (1 << 22) ||
        p.nsub < 1 || p.nshards % p.nsub || p.nshards / p.nsub > 32 || p.ag_parts < 1 ||
        p.ag_tab == nullptr || p.flag_rows * p.lda * esz / p.ag_parts >= (int64_t(1) << 30))
      return hipErrorNotSupported;  // (a copy unit is addressed by one 32-bit buffer descriptor)
    tile = TILE_PT4;
  } else if (p.ag_mode != 0) {
    return hipErrorNotSupported;  // agent-scope gate acquire only for flags this launch sets
  }
  if (mode < GEMM_MODE_AUTO || mode > GEMM_MODE_MX) return hipErrorInvalidValue;
  const bool fast = mode != GEMM_MODE_GENERIC && gemm_fast_path_ok(p, din, dout);
  if (p.tile_order && !fast) p.tile_order = 0;
  if (fast) {
    if (tile == TILE_AUTO) tile = choose_tile(p.M, p.N, p.K, din);
    if (p.nsub < 1) p.nsub = 1;
    if (p.tile_order && (p.nshards <= 0 || p.M % p.nshards != 0 || p.nshards % p.nsub != 0 ||
                         (p.M / p.nshards) % tile_rows(tile) != 0)) {
      // tile_order 3 also means "the own blocks are not gated": never drop it silently
      if (p.tile_order == 3) return hipErrorNotSupported;
      p.tile_order = 0;
    }
    if (p.tile_order == 2 && p.N % tile_cols(tile) != 0) p.tile_order = 0;  // whole tiles/shard
    hipError_t e = hipErrorInvalidValue;
    if (din == DT_FP8 && mode == GEMM_MODE_MX) e = launch_fast_mx(p, dout, tile, s);
    else e = launch_fast(p, din, dout, tile, s);
    if (e != hipErrorInvalidValue) return e;
  }
  if (p.flags != nullptr || p.c_table != nullptr)
    return hipErrorNotSupported;  // arrival flags / direct-store C need the tiled kernels
  return launch_generic(p, din, dout, s);
}

}  // namespace ddlb
