// Tile / work-unit index maps of the MFMA GEMM kernels, usable on the host too (host-side tests
// with sanitizers check that every map is a bijection: tests/native/test_tile_maps.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gemm.h"

namespace ddlb {

// Rows and group sizes fit in 32 bits: 32-bit unsigned division is ~10x cheaper than 64-bit.
__host__ __device__ inline int64_t map_row(int64_t i, int64_t grp, int64_t gstride) {
  const unsigned ui = (unsigned)i, ug = (unsigned)grp;
  const unsigned q = ui / ug;
  return (int64_t)q * gstride + (int64_t)(ui - q * ug);
}

// Bijective XCD remap (guide §5, "XCD swizzle must be bijective").
__host__ __device__ inline int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// Block -> tile. Default: bijective XCD remap over the whole grid. With ``tile_order`` the grid
// is dispatched shard-major (ordered_shard: the shard that arrives first runs first; with nsub > 1
// row blocks of all producers interleave block-major) and XCD-remapped within each shard;
// tile_order 2 interleaves the shards.
// ordered_shard: dispatch position j -> shard; producers rotate fastest (own first), blocks
// slowest.
// tile_order 3 (own first): the first producer's nsub blocks (the caller's own rows: a gated
// GEMM never waits for them, wait_flag_t0), then block-major over the other producers, rotating
// from first_shard + 1 (the order the stage collectives of an RCCL-fed gated GEMM deliver them).
// OWN_FIRST = false compiles tile_order 3 out (it then dispatches like 1): the ungated kernels
// never get it, and the extra branch cost the flagship kernel 11 spilled SGPRs.
template <bool OWN_FIRST = true>
__host__ __device__ inline int ordered_shard(const GemmArgs& p, int j) {
  const int np = p.nshards / p.nsub;
  if (OWN_FIRST && p.tile_order == 3) {
    if (j < p.nsub || np < 2) return p.first_shard * p.nsub + j;
    j -= p.nsub;
    return ((p.first_shard + 1 + j % (np - 1)) % np) * p.nsub + j / (np - 1);
  }
  return ((p.first_shard + j % np) % np) * p.nsub + j / np;
}

template <bool OWN_FIRST = true>
__host__ __device__ inline int tile_index_virtual(const GemmArgs& p, int vid, int nwg) {
  if (!p.tile_order) return xcd_remap(vid, nwg);
  if (p.tile_order == 2) {
    // shards interleaved: consecutive ids (one per XCD) walk different shards, so the tiles in
    // flight cover every shard at once (a direct-store GEMM keeps every peer's link busy) and,
    // with nshards dividing 8, each XCD stays on one shard (its A panels in that XCD's L2)
    const int ns = p.nshards, per = nwg / ns;
    return (vid % ns) * per + vid / ns;
  }
  const int per = nwg / p.nshards;
  const int j = vid / per, local = vid % per;
  return ordered_shard<OWN_FIRST>(p, j) * per + xcd_remap(local, per);
}

// Tile id -> (tm, tn). Row-major, except that without a shard order and with more than 4 column
// tiles, ids are rastered in groups of G = raster_g m-blocks (default 4, column-major inside a
// group): the 32 tiles an XCD runs together (consecutive ids after xcd_remap) then cover 4 m-blocks
// x 8 n-blocks, i.e. 12 A / B panels in its L2 instead of 1 + 32 (guide §5, L2 reuse per XCD).
// Measured (profiles/r03/r3_9_raster_*.txt, pt4, one box): 16384x8192x8192 G = 2 / 4 / 8 / 16:
// 1.430 / 1.395 / 1.465 / 1.451 ms; 8192^3 0.704 / 0.688 / 0.688 / 0.703 ms. Bijective for every
// G >= 1.
__host__ __device__ inline void tile_mn(const GemmArgs& p, int wg, int tiles_m, int tiles_n,
                                        int& tm, int& tn) {
  const int G = p.raster_g > 0 ? p.raster_g : 4;
  if (p.tile_order || tiles_n <= 4) {
    tm = wg / tiles_n;
    tn = wg % tiles_n;
    return;
  }
  const int per = G * tiles_n, grp = wg / per, first = grp * G;
  const int gs = tiles_m - first < G ? tiles_m - first : G, in = wg - grp * per;
  tm = first + in % gs;
  tn = in / gs;
}

// In-kernel all-gather work unit u -> (block b, producer prod, part pi): block-major; within a
// block, consecutive units go to different producers (ring order from rank + 1), so the copy
// workgroups in flight spread over every peer / xGMI link.
__host__ __device__ inline void ag_unit(int u, int np, int parts, int rank, int& b, int& prod,
                                        int& pi) {
  const int per_b = (np - 1) * parts;
  b = u / per_b;
  const int r = u % per_b;
  prod = (rank + 1 + r % (np - 1)) % np;
  pi = r / (np - 1);
}

// AG_FILL_ROUNDS: copy workgroups of a launch of `grid` workgroups whose GEMM part runs `tiles`
// tiles persistently: at least `ag` (rounded up to 8), grown while the GEMM's
// number of tile rounds ceil(tiles / gemm workgroups) stays the same.
inline int ag_fill_ctas(int grid, int ag, int tiles) {
  ag = (ag + 7) / 8 * 8;
  if (grid - ag < 8) return ag;
  const int g0 = (grid - ag) / 8 * 8;
  const int rounds = (tiles + g0 - 1) / g0;
  const int need = ((tiles + rounds - 1) / rounds + 7) / 8 * 8;
  return grid - need > ag ? (grid - need) / 8 * 8 : ag;
}

}  // namespace ddlb
