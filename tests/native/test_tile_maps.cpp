// Host-side checks of the GEMM's index maps (csrc/gemm/tile_map.h), built with
// AddressSanitizer + UndefinedBehaviorSanitizer on the host only (tests/test_native_host.py):
//  * tile_index_virtual is a bijection on [0, ntiles) for tile_order 0 / 1 / 2 / 3 and every
//    shard layout the plans use, tile_order 2 puts consecutive ids on different shards, and
//    tile_order 3 dispatches the first producer's blocks before any other producer's;
//  * tile_mn is a bijection onto the (tm, tn) grid (grouped raster included);
//  * the in-kernel all-gather's units cover every (block, producer != rank, part) exactly once,
//    and each run of np - 1 consecutive units of a block visits every peer;
//  * ag_fill_ctas never adds a GEMM tile round and never shrinks the copy role.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gemm/tile_map.h"

using ddlb::GemmArgs;

static int failures = 0;
#define CHECK(c, ...)                         \
  do {                                        \
    if (!(c)) {                               \
      ++failures;                             \
      std::fprintf(stderr, __VA_ARGS__);      \
      std::fprintf(stderr, "\n");             \
      if (failures > 20) std::exit(1);        \
    }                                         \
  } while (0)

static void check_tile_index(int ntiles, int order, int nshards, int nsub, int first) {
  GemmArgs p;
  p.tile_order = order;
  p.nshards = nshards;
  p.nsub = nsub;
  p.first_shard = first;
  std::vector<int> seen(ntiles, 0);
  for (int v = 0; v < ntiles; ++v) {
    const int t = ddlb::tile_index_virtual(p, v, ntiles);
    CHECK(t >= 0 && t < ntiles, "tile_index out of range: order %d ntiles %d v %d -> %d", order,
          ntiles, v, t);
    if (t >= 0 && t < ntiles) ++seen[t];
  }
  for (int t = 0; t < ntiles; ++t)
    CHECK(seen[t] == 1, "tile_index not bijective: order %d ntiles %d shards %d nsub %d tile %d x%d",
          order, ntiles, nshards, nsub, t, seen[t]);
  if (order == 2 && nshards > 1) {
    const int per = ntiles / nshards;
    for (int v = 0; v + 1 < ntiles && v + 1 < nshards; ++v)
      CHECK(ddlb::tile_index_virtual(p, v, ntiles) / per !=
                ddlb::tile_index_virtual(p, v + 1, ntiles) / per,
            "tile_order 2: ids %d, %d on one shard", v, v + 1);
  }
  if (order == 3) {
    const int per = ntiles / nshards;
    for (int v = 0; v < nsub * per; ++v)
      CHECK(ddlb::tile_index_virtual(p, v, ntiles) / per / nsub == first,
            "tile_order 3: id %d not in the first producer's blocks", v);
  }
}

static void check_tile_mn(int tm_n, int tn_n, int order, int g = 8) {
  GemmArgs p;
  p.tile_order = order;
  p.raster_g = g;
  std::vector<int> seen(tm_n * tn_n, 0);
  for (int w = 0; w < tm_n * tn_n; ++w) {
    int tm = -1, tn = -1;
    ddlb::tile_mn(p, w, tm_n, tn_n, tm, tn);
    CHECK(tm >= 0 && tm < tm_n && tn >= 0 && tn < tn_n, "tile_mn out of range %d -> %d,%d", w, tm,
          tn);
    if (tm >= 0 && tm < tm_n && tn >= 0 && tn < tn_n) ++seen[tm * tn_n + tn];
  }
  for (int i = 0; i < tm_n * tn_n; ++i)
    CHECK(seen[i] == 1, "tile_mn not bijective: %dx%d order %d G %d cell %d x%d", tm_n, tn_n, order,
          g, i, seen[i]);
}

static void check_ag_units(int np, int nsub, int parts, int rank) {
  const int units = nsub * (np - 1) * parts;
  std::vector<int> seen(nsub * np * parts, 0);
  for (int u = 0; u < units; ++u) {
    int b, prod, pi;
    ddlb::ag_unit(u, np, parts, rank, b, prod, pi);
    CHECK(b >= 0 && b < nsub && prod >= 0 && prod < np && prod != rank && pi >= 0 && pi < parts,
          "ag_unit out of range: np %d u %d -> b %d prod %d pi %d", np, u, b, prod, pi);
    if (b >= 0 && b < nsub && prod >= 0 && prod < np && pi >= 0 && pi < parts)
      ++seen[(b * np + prod) * parts + pi];
  }
  for (int b = 0; b < nsub; ++b)
    for (int q = 0; q < np; ++q)
      for (int i = 0; i < parts; ++i)
        CHECK(seen[(b * np + q) * parts + i] == (q == rank ? 0 : 1),
              "ag_unit coverage: np %d rank %d (b %d, prod %d, part %d) x%d", np, rank, b, q, i,
              seen[(b * np + q) * parts + i]);
  // every window of np - 1 consecutive units inside a block touches np - 1 distinct producers
  for (int u0 = 0; u0 + np - 1 <= units; u0 += np - 1) {
    std::vector<int> hit(np, 0);
    for (int u = u0; u < u0 + np - 1; ++u) {
      int b, prod, pi;
      ddlb::ag_unit(u, np, parts, rank, b, prod, pi);
      ++hit[prod];
    }
    for (int q = 0; q < np; ++q)
      CHECK(hit[q] == (q == rank ? 0 : 1), "ag_unit window at %d: producer %d x%d", u0, q, hit[q]);
  }
}

static void check_fill(int grid, int ag, int tiles) {
  const int base = (ag + 7) / 8 * 8;
  const int out = ddlb::ag_fill_ctas(grid, ag, tiles);
  CHECK(out >= base && out % 8 == 0, "ag_fill_ctas shrank / misaligned: %d %d %d -> %d", grid, ag,
        tiles, out);
  if (grid - base >= 8) {
    const int g0 = (grid - base) / 8 * 8, g1 = (grid - out) / 8 * 8;
    CHECK(g1 >= 8, "ag_fill_ctas left no GEMM workgroups: %d %d %d -> %d", grid, ag, tiles, out);
    if (g1 >= 8)
      CHECK((tiles + g1 - 1) / g1 == (tiles + g0 - 1) / g0,
            "ag_fill_ctas added a tile round: grid %d ag %d tiles %d -> %d", grid, ag, tiles, out);
  }
}

int main() {
  for (int ntiles : {8, 64, 96, 256, 1024, 2048, 4096})
    for (int order : {0, 1, 2, 3})
      for (int nshards : {1, 2, 3, 4, 6, 8, 16, 24, 32, 64})
        for (int nsub : {1, 2, 4, 8}) {
          if (ntiles % nshards || nshards % nsub) continue;
          if (order == 0 && (nshards != 1 || nsub != 1)) continue;
          if (order == 2 && nsub != 1) continue;
          for (int first = 0; first < nshards / nsub; first += (nshards / nsub > 3 ? 3 : 1))
            check_tile_index(ntiles, order, nshards, nsub, first);
        }
  for (int tm : {1, 3, 8, 13, 64, 256})
    for (int tn : {1, 2, 4, 5, 6, 32})
      for (int order : {0, 1})
        for (int g : {1, 2, 4, 8, 16, 0}) check_tile_mn(tm, tn, order, g);
  for (int np : {2, 3, 4, 8})
    for (int nsub : {1, 2, 8})
      for (int parts : {1, 3, 8})
        for (int rank = 0; rank < np; ++rank) check_ag_units(np, nsub, parts, rank);
  for (int grid : {64, 192, 224, 248, 256, 304})
    for (int ag : {1, 8, 16, 32, 48, 64})
      for (int tiles : {64, 256, 512, 1000, 1024, 2048, 4096}) check_fill(grid, ag, tiles);
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("tile maps ok\n");
  return 0;
}
