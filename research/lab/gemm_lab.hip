// Standalone GEMM lab (not part of the extension): iterate on new CDNA4 GEMM schedules with a
// plain executable, validate against an fp32 reference kernel, time with hipEvents.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 research/lab/gemm_lab.hip -o build/gemm_lab
//   build/gemm_lab 65536 1024 1024
//
// Kernel under test: "ring" — persistent 256x256 tiles, 8 waves (2x4, 128x64 per wave),
// K sliced in 32-deep steps (64-byte LDS rows), NS-slot LDS ring filled by LDS-DMA with
// NS-1 steps in flight ACROSS barriers (counted vmcnt, never 0 inside the stream), one raw
// barrier per step, C stores of tile i draining under tile i+1.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <type_traits>
#include <vector>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))

struct Args {
  const void* a;
  const void* b;
  void* c;
  int64_t lda, ldb, ldc;
  int M, N, K;
  unsigned long long* stamps;  // optional per-wave cycle breakdown
  int raster = 0;              // pt4v / pt4d: tile raster groups of this many m-blocks (product tile_mn)
};

// the product's tile raster (csrc/gemm/tile_map.h tile_mn, G m-blocks per group)
__device__ __forceinline__ void lab_tile_mn(int wg, int tiles_m, int tiles_n, int G, int64_t& m0,
                                            int64_t& n0) {
  if (G <= 0 || tiles_n <= 4) {
    m0 = (int64_t)(wg / tiles_n) * 256;
    n0 = (int64_t)(wg % tiles_n) * 256;
    return;
  }
  const int per = G * tiles_n, grp = wg / per, first = grp * G;
  const int gs = tiles_m - first < G ? tiles_m - first : G, in = wg - grp * per;
  m0 = (int64_t)(first + in % gs) * 256;
  n0 = (int64_t)(in / gs) * 256;
}

__device__ __forceinline__ void glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds((const GLB_AS void*)g, (LDS_AS void*)lds, 16, 0, 0);
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// swizzle of 16-byte chunk positions inside a 64-byte row: conflict-free ds_read_b128 for
// 16-row fragments (brute-forced against the gfx950 lane groups)
__device__ __forceinline__ int swz64(int row) { return (row >> 1) & 2; }

template <int NS, int DPOS, bool STAMP, int EPI = 0>
__global__ __launch_bounds__(512) void ring_kernel(const Args p) {
  constexpr int BM = 256, BN = 256, WN = 4;
  constexpr int ROWB = 64;  // bytes per row per K-step (32 bf16)
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, SLOT = A_BYTES + B_BYTES;
  constexpr int TM = 128, TN = 64, MR = TM / 16, NR = TN / 16;
  constexpr int LA = BM / 16 / 8, LB = BN / 16 / 8;  // DMA instructions per wave per step
  constexpr int NDMA = LA + LB;
  constexpr int NSTORE = EPI == 1 ? MR * NR / 2 : (EPI == 2 ? 0 : MR * NR);
  constexpr int NQ = MR * NR;
  __shared__ __attribute__((aligned(1024))) char smem[NS * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_n = p.N / BN, tiles_m = p.M / BM, ntiles = tiles_m * tiles_n;
  const int nk = p.K * 2 / ROWB;
  const int my_tiles =
      ((int)blockIdx.x < ntiles) ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int total = my_tiles * nk;
  if (total == 0) return;

  // DMA lane mapping: 16 rows x 64 B per instruction; lane -> (row l>>2, physical chunk l&3)
  const int drow = lane >> 2, dchunk = lane & 3;
  const char* abase[LA];
  const char* bbase[LB];
  int dma_tile = -1;
  auto set_dma_tile = [&](int ti) {
    const int wg = xcd_remap((int)blockIdx.x + ti * (int)gridDim.x, ntiles);
    const int64_t m0 = (int64_t)(wg / tiles_n) * BM, n0 = (int64_t)(wg % tiles_n) * BN;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int row = (wave * LA + i) * 16 + drow;
      abase[i] = (const char*)p.a + (m0 + row) * p.lda * 2 + ((dchunk ^ swz64(row)) * 16);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int row = (wave * LB + i) * 16 + drow;
      // EPI 1: LDS row t of each 32-row block holds column 8*((t&15)>>2) + 4*(t>>4) + (t&3), so a
      // lane's two adjacent fragments hold 8 consecutive columns (one 16-byte store)
      const int t32 = row & 31;
      const int gcol = EPI == 1 ? (row & ~31) + 8 * ((t32 & 15) >> 2) + 4 * (t32 >> 4) + (t32 & 3) : row;
      bbase[i] = (const char*)p.b + (n0 + gcol) * p.ldb * 2 + ((dchunk ^ swz64(row)) * 16);
    }
  };
  // DMA of stream step g (clamped to the last step: past the end a harmless duplicate lands in a
  // slot nobody reads again, which keeps the per-step vmcnt arithmetic uniform) into slot gs
  auto prep = [&](int g) -> int64_t {
    g = g < total ? g : total - 1;
    const int ti = g / nk;
    if (ti != dma_tile) {
      set_dma_tile(ti);
      dma_tile = ti;
    }
    return (int64_t)(g - ti * nk) * ROWB;
  };
  auto dma = [&](int d, int64_t koff, char* base) {
    if (d < LA) glds16(abase[d] + koff, base + (wave * LA + d) * 1024);
    else glds16(bbase[d - LA] + koff, base + A_BYTES + (wave * LB + d - LA) * 1024);
  };

  const int wm = wave / WN, wn = wave % WN;
  const int frow = lane & 15, fq = lane >> 4;
  const int rdoff = frow * ROWB + ((fq ^ swz64(frow)) * 16);
  f32x4 acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  unsigned long long t_wait = 0, t_bar = 0, t_comp = 0, t_epi = 0, t0 = 0, t1 = 0;

  // prologue: NS-1 steps in flight
  for (int g = 0; g < NS - 1; ++g) {
    const int64_t koff = prep(g);
#pragma unroll
    for (int d = 0; d < NDMA; ++d) dma(d, koff, smem + (g % NS) * SLOT);
  }

  int stores_window = 0;  // bit j: step (g-1-j) issued C stores (after DMA(g) in issue order)
  for (int g = 0; g < total; ++g) {
    if constexpr (STAMP) t0 = __builtin_readcyclecounter();
    // wait until step g's DMA landed: ops issued after it = DMA of steps g+1..g+NS-2 + the
    // stores of any tile that ended in steps g-NS+1..g-1
    const int nst = __builtin_popcount(stores_window);
    if (nst == 0) wait_vm<NDMA*(NS - 2)>();
    else if (nst == 1) wait_vm<(NDMA*(NS - 2) + NSTORE < 63 ? NDMA*(NS - 2) + NSTORE : 63)>();
    else wait_vm<(NDMA*(NS - 2) + 2 * NSTORE < 63 ? NDMA*(NS - 2) + 2 * NSTORE : 63)>();
    if constexpr (STAMP) { t1 = __builtin_readcyclecounter(); t_wait += t1 - t0; t0 = t1; }
    const int64_t koff = prep(g + NS - 1);
    char* nbase = smem + ((g + NS - 1) % NS) * SLOT;
    __builtin_amdgcn_s_barrier();
    if constexpr (STAMP) { t1 = __builtin_readcyclecounter(); t_bar += t1 - t0; t0 = t1; }

    const char* As = smem + (g % NS) * SLOT;
    const char* Bs = As + A_BYTES;
    if constexpr (DPOS == 0) {
#pragma unroll
      for (int d = 0; d < NDMA; ++d) dma(d, koff, nbase);
    }
    i32x4 af[MR], bfr[NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) bfr[j] = *(const i32x4*)(Bs + (wn * TN + j * 16) * ROWB + rdoff);
#pragma unroll
    for (int i = 0; i < MR; ++i) af[i] = *(const i32x4*)(As + (wm * TM + i * 16) * ROWB + rdoff);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int i = q / NR, j = q % NR;
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bfr[j]),
                                                          __builtin_bit_cast(bf16x8, af[i]),
                                                          acc[i][j], 0, 0, 0);
      if constexpr (DPOS == 1) {
        if (q == NQ / 2 - 1) {
#pragma unroll
          for (int d = 0; d < NDMA; ++d) dma(d, koff, nbase);
        }
      }
      if constexpr (DPOS == 2) {
        if (q % (NQ / NDMA) == 0) dma(q / (NQ / NDMA), koff, nbase);
      }
    }
    if constexpr (DPOS == 2) {
      __builtin_amdgcn_sched_group_barrier(0x100, MR + NR, 0);  // fragment reads first
#pragma unroll
      for (int d = 0; d < NDMA; ++d) {
        __builtin_amdgcn_sched_group_barrier(0x008, NQ / NDMA, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (STAMP) { t1 = __builtin_readcyclecounter(); t_comp += t1 - t0; t0 = t1; }

    const int ti = g / nk;
    const bool last_k = (g - ti * nk) == nk - 1;
    stores_window = (stores_window << 1) & ((1 << (NS - 1)) - 1);
    if (last_k) {
      const int wg = xcd_remap((int)blockIdx.x + ti * (int)gridDim.x, ntiles);
      const int64_t m0 = (int64_t)(wg / tiles_n) * BM, n0 = (int64_t)(wg % tiles_n) * BN;
      __builtin_amdgcn_sched_barrier(0);
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
      if constexpr (EPI == 0 || EPI == 2) {
        if (EPI == 0 || p.M < 0) {
#pragma unroll
          for (int i = 0; i < MR; ++i) {
            char* crow = (char*)p.c + (m0 + wm * TM + i * 16 + frow) * p.ldc * 2;
#pragma unroll
            for (int j = 0; j < NR; ++j) {
              const int64_t col = n0 + wn * TN + j * 16 + fq * 4;
              const f32x4 v = acc[i][j];
              bf16x4 o = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
              *(uint2*)(crow + col * 2) = __builtin_bit_cast(uint2, o);
            }
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < MR; ++i) {
          char* crow = (char*)p.c + (m0 + wm * TM + i * 16 + frow) * p.ldc * 2;
#pragma unroll
          for (int jp = 0; jp < NR / 2; ++jp) {
            const int64_t col = n0 + wn * TN + jp * 32 + fq * 8;
            const f32x4 v0 = acc[i][2 * jp], v1 = acc[i][2 * jp + 1];
            typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8o;
            bf16x8o o = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                         (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
            *(uint4*)(crow + col * 2) = __builtin_bit_cast(uint4, o);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      __builtin_amdgcn_sched_barrier(0);
      stores_window |= 1;
      if constexpr (STAMP) { t1 = __builtin_readcyclecounter(); t_epi += t1 - t0; t0 = t1; }
    }
  }
  wait_vm<0>();
  if constexpr (STAMP) {
    if (lane == 0) {
      unsigned long long* s = p.stamps + ((size_t)blockIdx.x * 8 + wave) * 4;
      s[0] = t_wait; s[1] = t_bar; s[2] = t_comp; s[3] = t_epi;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// ring2: same ring, but the barrier sits in the MIDDLE of a step's MFMAs so the matrix pipe never
// waits for fragment reads:
//   part A: MFMAs rows 0-3 (A0 x Bc) + DMA of step g+NS-1 + reads of A1 (rows 4-7, step g)
//   wait DMA(g+1); lgkmcnt(0); barrier
//   part C: MFMAs rows 4-7 (A1 x Bc) + reads of A0 and Bn for step g+1
template <int NS, bool STAMP, int DMAP = 0, int PRIO = 0, int EPI = 1, int SKIP = 0>
__global__ __launch_bounds__(512) void ring2_kernel(const Args p) {
  constexpr int BM = 256, BN = 256, WN = 4;
  constexpr int ROWB = 64;
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, SLOT = A_BYTES + B_BYTES;
  constexpr int TM = 128, TN = 64, MR = TM / 16, NR = TN / 16, MH = MR / 2;
  constexpr int LA = BM / 16 / 8, LB = BN / 16 / 8;
  constexpr int NDMA = LA + LB;
  constexpr int NSTORE = MR * NR / 2;  // 16-byte stores
  static_assert(NS >= 3, "need at least one step in flight beyond the next");
  __shared__ __attribute__((aligned(1024))) char smem[NS * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_n = p.N / BN, tiles_m = p.M / BM, ntiles = tiles_m * tiles_n;
  const int nk = p.K * 2 / ROWB;
  const int my_tiles =
      ((int)blockIdx.x < ntiles) ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int total = my_tiles * nk;
  if (total == 0) return;

  const int drow = lane >> 2, dchunk = lane & 3;
  bool g_loop_started = false;
  const char* abase[LA];
  const char* bbase[LB];
  int dma_tile = -1;
  auto set_dma_tile = [&](int ti) {
    const int wg = xcd_remap((int)blockIdx.x + ti * (int)gridDim.x, ntiles);
    const int64_t m0 = (int64_t)(wg / tiles_n) * BM, n0 = (int64_t)(wg % tiles_n) * BN;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int row = (wave * LA + i) * 16 + drow;
      abase[i] = (const char*)p.a + (m0 + row) * p.lda * 2 + ((dchunk ^ swz64(row)) * 16);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int row = (wave * LB + i) * 16 + drow;
      const int t32 = row & 31;
      const int gcol = (row & ~31) + 8 * ((t32 & 15) >> 2) + 4 * (t32 >> 4) + (t32 & 3);
      bbase[i] = (const char*)p.b + (n0 + gcol) * p.ldb * 2 + ((dchunk ^ swz64(row)) * 16);
    }
  };
  auto prep = [&](int g) -> int64_t {
    g = g < total ? g : total - 1;
    const int ti = g / nk;
    if (ti != dma_tile) {
      set_dma_tile(ti);
      dma_tile = ti;
    }
    return (int64_t)(g - ti * nk) * ROWB;
  };
  auto dma = [&](int d, int64_t koff, char* base) {
    if ((SKIP & 1) && koff >= 0 && p.M > 0 && dma_tile >= 0 && base != smem - 1) {
      if (g_loop_started) return;
    }
    if (d < LA) glds16(abase[d] + koff, base + (wave * LA + d) * 1024);
    else glds16(bbase[d - LA] + koff, base + A_BYTES + (wave * LB + d - LA) * 1024);
  };

  const int wm = wave / WN, wn = wave % WN;
  const int frow = lane & 15, fq = lane >> 4;
  const int rdoff = frow * ROWB + ((fq ^ swz64(frow)) * 16);
  const int aoff = wm * TM * ROWB + rdoff, boff = A_BYTES + wn * TN * ROWB + rdoff;
  f32x4 acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](int i, int j, const i32x4& a, const i32x4& b) {
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, b),
                                                        __builtin_bit_cast(bf16x8, a), acc[i][j],
                                                        0, 0, 0);
  };

  unsigned long long t_wait = 0, t_a = 0, t_c = 0, t_epi = 0, t_vm = 0, t0 = 0, t1 = 0;
  unsigned long long c_start = 0, r_start = 0;
  if constexpr (STAMP) {
    c_start = __builtin_readcyclecounter();
    r_start = __builtin_amdgcn_s_memrealtime();
  }

  for (int g = 0; g < NS - 1; ++g) {
    const int64_t koff = prep(g);
#pragma unroll
    for (int d = 0; d < NDMA; ++d) dma(d, koff, smem + (g % NS) * SLOT);
  }
  wait_vm<NDMA*(NS - 2)>();
  __builtin_amdgcn_s_barrier();
  i32x4 A0[MH], A1[MH], Bc[NR], Bn[NR];
  if constexpr ((SKIP & 4) != 0) {
#pragma unroll
    for (int i = 0; i < MH; ++i) A1[i] = *(const i32x4*)(smem + aoff + (MH + i) * 16 * ROWB);
#pragma unroll
    for (int j = 0; j < NR; ++j) Bn[j] = *(const i32x4*)(smem + boff + j * 16 * ROWB);
  }
#pragma unroll
  for (int j = 0; j < NR; ++j) Bc[j] = *(const i32x4*)(smem + boff + j * 16 * ROWB);
#pragma unroll
  for (int i = 0; i < MH; ++i) A0[i] = *(const i32x4*)(smem + aoff + i * 16 * ROWB);

  if constexpr (PRIO == 1) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  }
  int stores_window = 0;  // bit j: step g-1-j issued C stores
  g_loop_started = true;
  for (int g = 0; g < total; ++g) {
    if constexpr (STAMP) t0 = __builtin_readcyclecounter();
    const char* cur = smem + (g % NS) * SLOT;
    const char* nxt = smem + ((g + 1) % NS) * SLOT;
    const int64_t koff = prep(g + NS - 1);
    char* nbase = smem + ((g + NS - 1) % NS) * SLOT;
    // ---- part A
    constexpr int DA = DMAP == 0 ? NDMA : (DMAP == 1 ? 0 : NDMA / 2);  // DMAs in part A
    if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < MH * NR; ++q) {
      const int i = q / NR, j = q % NR;
      mma(i, j, A0[i], Bc[j]);
      if (DA > 0 && q % (16 / (DA > 0 ? DA : 1)) == 1) dma(q / (16 / (DA > 0 ? DA : 1)), koff, nbase);
      if (!(SKIP & 4) && q % 4 == 3) A1[q / 4] = *(const i32x4*)(cur + aoff + (MH + q / 4) * 16 * ROWB);
    }
    if constexpr (DA == 4) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    } else if constexpr (DA == 2) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    }
    if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(0);
    if constexpr (STAMP) { t1 = __builtin_readcyclecounter(); t_a += t1 - t0; t0 = t1; }
    // ---- wait for step g+1's DMA (ops issued after it: DMA of g+2..g+NS-1, stores of steps
    //      g-NS+2..g-1), all fragment reads of this slot done, barrier
    // DMA halves issued in part C of step g-NS+2 are the newest part of DMA(g+1)
    constexpr int VMB = NDMA * (NS - 2) - (NDMA - DA);
    const int nst = __builtin_popcount(stores_window);
    if (nst == 0) wait_vm<VMB>();
    else if (nst == 1) wait_vm<(VMB + NSTORE < 63 ? VMB + NSTORE : 63)>();
    else wait_vm<(VMB + 2 * NSTORE < 63 ? VMB + 2 * NSTORE : 63)>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (STAMP) { t1 = __builtin_readcyclecounter(); t_vm += t1 - t0; t0 = t1; }
    if constexpr (!(SKIP & 2)) __builtin_amdgcn_s_barrier();
    if constexpr (STAMP) { t1 = __builtin_readcyclecounter(); t_wait += t1 - t0; t0 = t1; }
    // ---- part C
    constexpr int DC = NDMA - DA;
    if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < MH * NR; ++q) {
      const int j = q / MH, i = MH + q % MH;  // j-major: Bc[j] free after its 4 MFMAs
      mma(i, j, A1[i - MH], Bc[j]);
      if (q % 2 == 1) {
        const int r = q / 2;  // 8 reads: Bn[0..3], A0[0..3] of step g+1
        if (!(SKIP & 4)) {
          if (r < NR) Bn[r] = *(const i32x4*)(nxt + boff + r * 16 * ROWB);
          else A0[r - NR] = *(const i32x4*)(nxt + aoff + (r - NR) * 16 * ROWB);
        }
      }
      if (DC > 0 && q % (16 / (DC > 0 ? DC : 1)) == 0) dma(DA + q / (16 / (DC > 0 ? DC : 1)), koff, nbase);
    }
    if constexpr (DC == 0) {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        if ((r * 2) % (16 / (DC > 0 ? DC : 1)) == 0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    }
    if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(0);
    if constexpr (STAMP) { t1 = __builtin_readcyclecounter(); t_c += t1 - t0; t0 = t1; }
#pragma unroll
    for (int j = 0; j < NR; ++j) Bc[j] = Bn[j];

    const int ti = g / nk;
    const bool last_k = (g - ti * nk) == nk - 1;
    stores_window = (stores_window << 1) & ((1 << (NS - 2)) - 1);
    if (last_k) {
      const int wg = xcd_remap((int)blockIdx.x + ti * (int)gridDim.x, ntiles);
      const int64_t m0 = (int64_t)(wg / tiles_n) * BM, n0 = (int64_t)(wg % tiles_n) * BN;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        char* crow = (char*)p.c + (m0 + wm * TM + i * 16 + frow) * p.ldc * 2;
#pragma unroll
        for (int jp = 0; jp < NR / 2; ++jp) {
          const int64_t col = n0 + wn * TN + jp * 32 + fq * 8;
          const f32x4 v0 = acc[i][2 * jp], v1 = acc[i][2 * jp + 1];
          typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8o;
          bf16x8o o = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                       (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
          if (EPI == 3) __builtin_nontemporal_store(__builtin_bit_cast(i32x4, o), (i32x4*)(crow + col * 2));
          else if (EPI == 1 || p.M < 0) *(uint4*)(crow + col * 2) = __builtin_bit_cast(uint4, o);
        }
      }
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      __builtin_amdgcn_sched_barrier(0);
      stores_window |= 1;
      if constexpr (STAMP) { t1 = __builtin_readcyclecounter(); t_epi += t1 - t0; t0 = t1; }
    }
  }
  wait_vm<0>();
  if constexpr (STAMP) {
    if (lane == 0 && blockIdx.x == 0 && wave == 0) {
      p.stamps[(size_t)gridDim.x * 8 * 5 + 1] = __builtin_readcyclecounter() - c_start;
      p.stamps[(size_t)gridDim.x * 8 * 5 + 3] = __builtin_amdgcn_s_memrealtime() - r_start;
    }
    if (lane == 0) {
      unsigned long long* s = p.stamps + ((size_t)blockIdx.x * 8 + wave) * 5;
      s[0] = t_wait; s[1] = t_a; s[2] = t_c; s[3] = t_epi; s[4] = t_vm;
    }
  }
}

// 4-wave variant: 2x2 waves of 128x128 (one wave per SIMD, 256 accumulator registers)
template <int NS, bool STAMP, int DMAP = 2, int PRIO = 0, int EPI = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void ring4w_kernel(const Args p) {
  constexpr int BM = 256, BN = 256, WN = 2, NWAVE = 4;
  constexpr int ROWB = 64;
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, SLOT = A_BYTES + B_BYTES;
  constexpr int TM = 128, TN = 128, MR = TM / 16, NR = TN / 16, MH = MR / 2;
  constexpr int LA = BM / 16 / NWAVE, LB = BN / 16 / NWAVE;
  constexpr int NDMA = LA + LB;
  constexpr int NSTORE = MR * NR / 2;  // 16-byte stores
  static_assert(NS >= 3, "need at least one step in flight beyond the next");
  __shared__ __attribute__((aligned(1024))) char smem[NS * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_n = p.N / BN, tiles_m = p.M / BM, ntiles = tiles_m * tiles_n;
  const int nk = p.K * 2 / ROWB;
  const int my_tiles =
      ((int)blockIdx.x < ntiles) ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int total = my_tiles * nk;
  if (total == 0) return;

  const int drow = lane >> 2, dchunk = lane & 3;
  const char* abase[LA];
  const char* bbase[LB];
  int dma_tile = -1;
  auto set_dma_tile = [&](int ti) {
    const int wg = xcd_remap((int)blockIdx.x + ti * (int)gridDim.x, ntiles);
    const int64_t m0 = (int64_t)(wg / tiles_n) * BM, n0 = (int64_t)(wg % tiles_n) * BN;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int row = (wave * LA + i) * 16 + drow;
      abase[i] = (const char*)p.a + (m0 + row) * p.lda * 2 + ((dchunk ^ swz64(row)) * 16);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int row = (wave * LB + i) * 16 + drow;
      const int t32 = row & 31;
      const int gcol = (row & ~31) + 8 * ((t32 & 15) >> 2) + 4 * (t32 >> 4) + (t32 & 3);
      bbase[i] = (const char*)p.b + (n0 + gcol) * p.ldb * 2 + ((dchunk ^ swz64(row)) * 16);
    }
  };
  auto prep = [&](int g) -> int64_t {
    g = g < total ? g : total - 1;
    const int ti = g / nk;
    if (ti != dma_tile) {
      set_dma_tile(ti);
      dma_tile = ti;
    }
    return (int64_t)(g - ti * nk) * ROWB;
  };
  auto dma = [&](int d, int64_t koff, char* base) {
    if (d < LA) glds16(abase[d] + koff, base + (wave * LA + d) * 1024);
    else glds16(bbase[d - LA] + koff, base + A_BYTES + (wave * LB + d - LA) * 1024);
  };

  const int wm = wave / WN, wn = wave % WN;
  const int frow = lane & 15, fq = lane >> 4;
  const int rdoff = frow * ROWB + ((fq ^ swz64(frow)) * 16);
  const int aoff = wm * TM * ROWB + rdoff, boff = A_BYTES + wn * TN * ROWB + rdoff;
  f32x4 acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](int i, int j, const i32x4& a, const i32x4& b) {
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, b),
                                                        __builtin_bit_cast(bf16x8, a), acc[i][j],
                                                        0, 0, 0);
  };

  unsigned long long t_wait = 0, t_a = 0, t_c = 0, t_epi = 0, t_vm = 0, t0 = 0, t1 = 0;
  unsigned long long c_start = 0, r_start = 0;
  if constexpr (STAMP) {
    c_start = __builtin_readcyclecounter();
    r_start = __builtin_amdgcn_s_memrealtime();
  }

  for (int g = 0; g < NS - 1; ++g) {
    const int64_t koff = prep(g);
#pragma unroll
    for (int d = 0; d < NDMA; ++d) dma(d, koff, smem + (g % NS) * SLOT);
  }
  wait_vm<NDMA*(NS - 2)>();
  __builtin_amdgcn_s_barrier();
  i32x4 A0[MH], A1[MH], Bc[NR], Bn[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) Bc[j] = *(const i32x4*)(smem + boff + j * 16 * ROWB);
#pragma unroll
  for (int i = 0; i < MH; ++i) A0[i] = *(const i32x4*)(smem + aoff + i * 16 * ROWB);

  if constexpr (PRIO == 1) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 128) __builtin_amdgcn_s_setprio(1);
  }
  int stores_window = 0;  // bit j: step g-1-j issued C stores
  for (int g = 0; g < total; ++g) {
    if constexpr (STAMP) t0 = __builtin_readcyclecounter();
    const char* cur = smem + (g % NS) * SLOT;
    const char* nxt = smem + ((g + 1) % NS) * SLOT;
    const int64_t koff = prep(g + NS - 1);
    char* nbase = smem + ((g + NS - 1) % NS) * SLOT;
    // ---- part A
    constexpr int DA = NDMA / 2;  // DMAs in part A
    if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < MH * NR; ++q) {
      const int i = q / NR, j = q % NR;
      mma(i, j, A0[i], Bc[j]);
      if (q % 8 == 1) dma(q / 8, koff, nbase);
      if (q % 8 == 5) A1[q / 8] = *(const i32x4*)(cur + aoff + (MH + q / 8) * 16 * ROWB);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(0);
    if constexpr (STAMP) { t1 = __builtin_readcyclecounter(); t_a += t1 - t0; t0 = t1; }
    // ---- wait for step g+1's DMA (ops issued after it: DMA of g+2..g+NS-1, stores of steps
    //      g-NS+2..g-1), all fragment reads of this slot done, barrier
    // DMA halves issued in part C of step g-NS+2 are the newest part of DMA(g+1)
    constexpr int VMB = NDMA * (NS - 2) - (NDMA - DA);
    const int nst = __builtin_popcount(stores_window);
    if (nst == 0) wait_vm<VMB>();
    else if (nst == 1) wait_vm<(VMB + NSTORE < 63 ? VMB + NSTORE : 63)>();
    else wait_vm<(VMB + 2 * NSTORE < 63 ? VMB + 2 * NSTORE : 63)>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (STAMP) { t1 = __builtin_readcyclecounter(); t_vm += t1 - t0; t0 = t1; }
    __builtin_amdgcn_s_barrier();
    if constexpr (STAMP) { t1 = __builtin_readcyclecounter(); t_wait += t1 - t0; t0 = t1; }
    // ---- part C
    if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < MH * NR; ++q) {
      const int j = q / MH, i = MH + q % MH;  // j-major: Bc[j] is free after its 4 MFMAs
      mma(i, j, A1[i - MH], Bc[j]);
      if (q % 4 == 3 && q / 4 < NR) Bn[q / 4] = *(const i32x4*)(nxt + boff + (q / 4) * 16 * ROWB);
      if (q % 8 == 1) A0[q / 8] = *(const i32x4*)(nxt + aoff + (q / 8) * 16 * ROWB);
      if (q % 8 == 5) dma(DA + q / 8, koff, nbase);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    if constexpr (PRIO == 0) __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (int j = 0; j < NR; ++j) Bc[j] = Bn[j];

    const int ti = g / nk;
    const bool last_k = (g - ti * nk) == nk - 1;
    stores_window = (stores_window << 1) & ((1 << (NS - 2)) - 1);
    if (last_k) {
      const int wg = xcd_remap((int)blockIdx.x + ti * (int)gridDim.x, ntiles);
      const int64_t m0 = (int64_t)(wg / tiles_n) * BM, n0 = (int64_t)(wg % tiles_n) * BN;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        char* crow = (char*)p.c + (m0 + wm * TM + i * 16 + frow) * p.ldc * 2;
#pragma unroll
        for (int jp = 0; jp < NR / 2; ++jp) {
          const int64_t col = n0 + wn * TN + jp * 32 + fq * 8;
          const f32x4 v0 = acc[i][2 * jp], v1 = acc[i][2 * jp + 1];
          typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8o;
          bf16x8o o = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                       (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
          if (EPI == 3) __builtin_nontemporal_store(__builtin_bit_cast(i32x4, o), (i32x4*)(crow + col * 2));
          else if (EPI == 1 || p.M < 0) *(uint4*)(crow + col * 2) = __builtin_bit_cast(uint4, o);
        }
      }
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      __builtin_amdgcn_sched_barrier(0);
      stores_window |= 1;
      if constexpr (STAMP) { t1 = __builtin_readcyclecounter(); t_epi += t1 - t0; t0 = t1; }
    }
  }
  wait_vm<0>();
  if constexpr (STAMP) {
    if (lane == 0 && blockIdx.x == 0 && wave == 0) {
      p.stamps[(size_t)gridDim.x * 8 * 5 + 1] = __builtin_readcyclecounter() - c_start;
      p.stamps[(size_t)gridDim.x * 8 * 5 + 3] = __builtin_amdgcn_s_memrealtime() - r_start;
    }
    if (lane == 0) {
      unsigned long long* s = p.stamps + ((size_t)blockIdx.x * 8 + wave) * 5;
      s[0] = t_wait; s[1] = t_a; s[2] = t_c; s[3] = t_epi; s[4] = t_vm;
    }
  }
}


// ---------------------------------------------------------------------------------------------
// t8: 256x256 tile, BK = 64 (128-byte LDS rows), 8 waves = 2 groups (wr) x 4 (wc), 128x64 per
// wave as 2x2 quadrants of 64x32 (cdna guide §5 "256^2 8-phase template": T2+T3+T4+T5).
// Group 1 runs one barrier behind group 0, so between any two barriers one group issues its
// ds_reads / LDS-DMA while the other runs 16 MFMAs. K-tile data moves in 16 KB units of 128 rows:
//   UA0 = A rows {0-63, 128-191} (quadrant row mq=0 of both groups), UA1 = {64-127, 192-255},
//   UB0 = B rows {wc*64 + 0..31}, UB1 = {wc*64 + 32..63};
// wave w stages unit rows [16w, 16w+16) (2 x 1 KB LDS-DMA). Per K-tile t (buffer t&1), phase p of
// a group reads / stages (intervals I_k between barriers; group g reads in I_{8t+2p+g}):
//   p0: read A(mq0) + B(nq0), stage UA1(t+1)   p1: read B(nq1), stage UB0(t+1)
//   p2: read A(mq1),          stage UA0(t+2)   p3: read B(nq0), stage UB1(t+2), vmcnt(4)
// RAW: vmcnt(4) (2 unit slices in flight) before barrier 8(t+1) retires every slice of K-tile t+1
// on every wave (group 1 in its p3 read section, group 0 after its p3 MFMAs).
// WAR: each unit is restaged 3 intervals after its last read (reads retire by lgkmcnt(0) in the
// next interval), e.g. UA0 of t read in I_{8t}, I_{8t+1}, restaged in I_{8t+4}, I_{8t+5}.
// Past the last K-tile the stage source is clamped to K-tile nk-1: identical bytes into units no
// one reads again, so the vmcnt arithmetic stays uniform.
__device__ __forceinline__ int t8_perm(int t) { return 8 * ((t & 15) >> 2) + 4 * (t >> 4) + (t & 3); }

template <bool STAMP>
__global__ __launch_bounds__(512) void t8_kernel(const Args p) {
  constexpr int ROWB = 128, UNIT = 128 * ROWB, STAGE = 4 * UNIT;
  constexpr int UA0 = 0, UA1 = UNIT, UB0 = 2 * UNIT, UB1 = 3 * UNIT;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int wg = xcd_remap((int)blockIdx.x, ntiles);
  const int64_t m0 = (int64_t)(wg / tiles_n) * 256, n0 = (int64_t)(wg % tiles_n) * 256;
  const int nk = p.K / 64;

  // ---- LDS-DMA sources of this wave's slices (2 instructions x 8 rows per unit)
  const int drow = lane >> 3, dpc = lane & 7;
  const char* sA[2][2];
  const char* sB[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ur = wave * 16 + i * 8 + drow;
    const int ch = (dpc ^ ((ur >> 1) & 7)) * 16;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int lr = (ur >> 6) * 128 + q * 64 + (ur & 63);
      sA[q][i] = (const char*)p.a + (m0 + lr) * p.lda * 2 + ch;
      const int lc = (ur >> 5) * 64 + q * 32 + t8_perm(ur & 31);
      sB[q][i] = (const char*)p.b + (n0 + lc) * p.ldb * 2 + ch;
    }
  }
  auto stage = [&](const char* const* src, int unit_off, int kt, int buf) {
    kt = kt < nk ? kt : nk - 1;
    char* dst = smem + buf * STAGE + unit_off + wave * 16 * ROWB;
    glds16(src[0] + (int64_t)kt * ROWB, dst);
    glds16(src[1] + (int64_t)kt * ROWB, dst + 8 * ROWB);
  };

  // ---- fragment reads: lane -> unit row base + (lane & 15), logical chunk kk*4 + (lane >> 4)
  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;
  const int c0 = ((0 + fq) ^ sw) * 16, c1 = ((4 + fq) ^ sw) * 16;
  const int aoff = (wr * 64 + frow) * ROWB, boff = (wc * 32 + frow) * ROWB;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x4 aR[4][2], bR[2][2];
  auto loadA = [&](const char* base, int mq) {
    const char* r = base + (mq ? UA1 : UA0) + aoff;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      aR[f][0] = *(const i32x4*)(r + f * 16 * ROWB + c0);
      aR[f][1] = *(const i32x4*)(r + f * 16 * ROWB + c1);
    }
  };
  auto loadB = [&](const char* base, int nq) {
    const char* r = base + (nq ? UB1 : UB0) + boff;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      bR[g][0] = *(const i32x4*)(r + g * 16 * ROWB + c0);
      bR[g][1] = *(const i32x4*)(r + g * 16 * ROWB + c1);
    }
  };
  auto comp = [&](int mq, int nq) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g)
          acc[mq * 4 + f][nq * 2 + g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, bR[g][kk]), __builtin_bit_cast(bf16x8, aR[f][kk]),
              acc[mq * 4 + f][nq * 2 + g], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
#define T8_BAR()                         \
  do {                                   \
    __builtin_amdgcn_sched_barrier(0);   \
    __builtin_amdgcn_s_barrier();        \
    __builtin_amdgcn_sched_barrier(0);   \
  } while (0)

  // ---- prologue: K-tile 0 whole, UA0 / UB1 of K-tile 1 in flight
  stage(sA[0], UA0, 0, 0);
  stage(sB[1], UB1, 0, 0);
  stage(sA[1], UA1, 0, 0);
  stage(sB[0], UB0, 0, 0);
  stage(sA[0], UA0, 1, 1);
  stage(sB[1], UB1, 1, 1);
  wait_vm<4>();
  T8_BAR();
  const bool g1 = wr == 1;  // wave-uniform
  if (g1) T8_BAR();
  for (int t = 0; t < nk; ++t) {
    const int b = t & 1, nb = b ^ 1;
    const char* cur = smem + b * STAGE;
    // p0
    loadA(cur, 0);
    loadB(cur, 0);
    stage(sA[1], UA1, t + 1, nb);
    T8_BAR();
    comp(0, 0);
    T8_BAR();
    // p1
    loadB(cur, 1);
    stage(sB[0], UB0, t + 1, nb);
    T8_BAR();
    comp(0, 1);
    T8_BAR();
    // p2
    loadA(cur, 1);
    stage(sA[0], UA0, t + 2, b);
    T8_BAR();
    comp(1, 1);
    T8_BAR();
    // p3
    loadB(cur, 0);
    stage(sB[1], UB1, t + 2, b);
    if (g1) wait_vm<4>();
    T8_BAR();
    comp(1, 0);
    if (!g1) wait_vm<4>();
    T8_BAR();
  }
  if (!g1) T8_BAR();
#undef T8_BAR
  wait_vm<0>();
  // ---- epilogue: lane holds columns 8*fq .. 8*fq+7 of each 32-column quadrant (B rows permuted)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    char* crow = (char*)p.c + (m0 + wr * 128 + (i >> 2) * 64 + (i & 3) * 16 + frow) * p.ldc * 2;
#pragma unroll
    for (int nq = 0; nq < 2; ++nq) {
      const f32x4 v0 = acc[i][nq * 2], v1 = acc[i][nq * 2 + 1];
      bf16x8 o = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                  (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
      *(uint4*)(crow + (n0 + wc * 64 + nq * 32 + fq * 8) * 2) = __builtin_bit_cast(uint4, o);
    }
  }
}


// pt8: persistent t8. One workgroup per CU streams its tiles' K-tiles back to back (stream index
// h = tile * nk + kt; the unit schedule of t8 runs across tile boundaries, so only the first tile
// pays the ring fill). A tile's C quadrants are stored right after their last MFMAs (quadrant
// (0,0) in phase 0 of the tile's last K-tile, ..., (1,0) in phase 3), spreading the C burst over
// a K-tile; stores issued after the UB0 stage of that K-tile stay in flight across its vmcnt.
template <bool STAMP>
__global__ __launch_bounds__(512) void pt8_kernel(const Args p) {
  constexpr int ROWB = 128, UNIT = 128 * ROWB, STAGE = 4 * UNIT;
  constexpr int UA0 = 0, UA1 = UNIT, UB0 = 2 * UNIT, UB1 = 3 * UNIT;
  constexpr int NS = 4;  // 16-byte C stores per quadrant per wave (bf16 out)
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int nk = p.K / 64;
  const int my_tiles =
      ((int)blockIdx.x < ntiles) ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int total = my_tiles * nk;
  if (total == 0) return;

  const int drow = lane >> 3, dpc = lane & 7;
  const char* sA[2][2];
  const char* sB[2][2];
  int src_tile = -1;
  auto set_src = [&](int ti) {
    const int wg = xcd_remap((int)blockIdx.x + ti * (int)gridDim.x, ntiles);
    const int64_t m0 = (int64_t)(wg / tiles_n) * 256, n0 = (int64_t)(wg % tiles_n) * 256;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ur = wave * 16 + i * 8 + drow;
      const int ch = (dpc ^ ((ur >> 1) & 7)) * 16;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int lr = (ur >> 6) * 128 + q * 64 + (ur & 63);
        sA[q][i] = (const char*)p.a + (m0 + lr) * p.lda * 2 + ch;
        const int lc = (ur >> 5) * 64 + q * 32 + t8_perm(ur & 31);
        sB[q][i] = (const char*)p.b + (n0 + lc) * p.ldb * 2 + ch;
      }
    }
  };
  // stage stream cursors (no integer division in the loop): (ti, kt) of h+1 and h+2, clamped
  // to the last K-tile of the last tile past the end of the stream
  struct Cur { int ti, kt; };
  auto adv = [&](Cur& c) {
    if (c.ti == my_tiles - 1 && c.kt == nk - 1) return;
    if (++c.kt == nk) { c.kt = 0; ++c.ti; }
  };
  auto stage = [&](int which, int unit_off, Cur c, int buf) {  // which: 0 A mq0, 1 A mq1, 2 B nq0, 3 B nq1
    const int ti = c.ti, kt = c.kt;
    if (ti != src_tile) {
      set_src(ti);
      src_tile = ti;
    }
    const char* const* src = which < 2 ? sA[which] : sB[which - 2];
    char* dst = smem + buf * STAGE + unit_off + wave * 16 * ROWB;
    glds16(src[0] + (int64_t)kt * ROWB, dst);
    glds16(src[1] + (int64_t)kt * ROWB, dst + 8 * ROWB);
  };

  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;
  const int c0 = ((0 + fq) ^ sw) * 16, c1 = ((4 + fq) ^ sw) * 16;
  const int aoff = (wr * 64 + frow) * ROWB, boff = (wc * 32 + frow) * ROWB;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x4 aR[4][2], bR[2][2];
  auto loadA = [&](const char* base, int mq) {
    const char* r = base + (mq ? UA1 : UA0) + aoff;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      aR[f][0] = *(const i32x4*)(r + f * 16 * ROWB + c0);
      aR[f][1] = *(const i32x4*)(r + f * 16 * ROWB + c1);
    }
  };
  auto loadB = [&](const char* base, int nq) {
    const char* r = base + (nq ? UB1 : UB0) + boff;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      bR[g][0] = *(const i32x4*)(r + g * 16 * ROWB + c0);
      bR[g][1] = *(const i32x4*)(r + g * 16 * ROWB + c1);
    }
  };
  auto comp = [&](int mq, int nq) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g)
          acc[mq * 4 + f][nq * 2 + g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, bR[g][kk]), __builtin_bit_cast(bf16x8, aR[f][kk]),
              acc[mq * 4 + f][nq * 2 + g], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // store + clear quadrant (mq, nq) of tile ti
  auto store_q = [&](int ti, int mq, int nq) {
    const int wg = xcd_remap((int)blockIdx.x + ti * (int)gridDim.x, ntiles);
    const int64_t m0 = (int64_t)(wg / tiles_n) * 256, n0 = (int64_t)(wg % tiles_n) * 256;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int i = mq * 4 + f;
      char* crow = (char*)p.c + (m0 + wr * 128 + mq * 64 + f * 16 + frow) * p.ldc * 2;
      const f32x4 v0 = acc[i][nq * 2], v1 = acc[i][nq * 2 + 1];
      bf16x8 o = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                  (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
      *(uint4*)(crow + (n0 + wc * 64 + nq * 32 + fq * 8) * 2) = __builtin_bit_cast(uint4, o);
      acc[i][nq * 2] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc[i][nq * 2 + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __builtin_amdgcn_sched_barrier(0);
  };
#define T8_BAR()                         \
  do {                                   \
    __builtin_amdgcn_sched_barrier(0);   \
    __builtin_amdgcn_s_barrier();        \
    __builtin_amdgcn_sched_barrier(0);   \
  } while (0)

  Cur q0{0, 0}, q1{0, 0};
  adv(q1);  // q0 = h, q1 = h + 1 (clamped)
  stage(0, UA0, q0, 0);
  stage(3, UB1, q0, 0);
  stage(1, UA1, q0, 0);
  stage(2, UB0, q0, 0);
  stage(0, UA0, q1, 1);
  stage(3, UB1, q1, 1);
  Cur q2 = q1;
  adv(q2);  // h + 2
  int ti = 0;
  wait_vm<4>();
  T8_BAR();
  const bool g1 = wr == 1;
  if (g1) T8_BAR();
  // one K-tile of the stream; LAST = the tile's last K-tile (stores its quadrants)
  auto iter = [&](int h, auto last_tag) {
    constexpr bool LAST = decltype(last_tag)::value;
    const int b = h & 1, nb = b ^ 1;
    const char* cur = smem + b * STAGE;
    loadA(cur, 0);  // p0
    loadB(cur, 0);
    stage(1, UA1, q1, nb);
    T8_BAR();
    comp(0, 0);
    if constexpr (LAST) store_q(ti, 0, 0);
    T8_BAR();
    loadB(cur, 1);  // p1
    stage(2, UB0, q1, nb);
    T8_BAR();
    comp(0, 1);
    if constexpr (LAST) store_q(ti, 0, 1);
    T8_BAR();
    loadA(cur, 1);  // p2
    stage(0, UA0, q2, b);
    T8_BAR();
    comp(1, 1);
    if constexpr (LAST) store_q(ti, 1, 1);
    T8_BAR();
    loadB(cur, 0);  // p3
    stage(3, UB1, q2, b);
    if (g1) wait_vm<LAST ? 4 + 2 * NS : 4>();  // younger than UB0(h+1): UA0/UB1(h+2), Q01, Q11
    T8_BAR();
    comp(1, 0);
    if constexpr (LAST) store_q(ti, 1, 0);
    if (!g1) wait_vm<LAST ? 4 + 3 * NS : 4>();  // ... and Q10
    T8_BAR();
    q1 = q2;
    adv(q2);
  };
  int h = 0;
  for (ti = 0; ti < my_tiles; ++ti) {
    for (int t = 0; t < nk - 1; ++t, ++h) iter(h, std::integral_constant<bool, false>{});
    iter(h, std::integral_constant<bool, true>{});
    ++h;
  }
  if (!g1) T8_BAR();
#undef T8_BAR
  wait_vm<0>();
}


// t8b: t8 with balanced fragment reads and a deeper staging pipeline. B0 of the NEXT K-tile is
// prefetched into registers in phase 3, so the phases read 8 / 4 / 8 / 4 fragments (A0 | B1 |
// A1 | B0') instead of 12 / 4 / 8 / 4, and the units are staged as soon as they free up:
//   p0: stage UA1(t+1)   p1: stage UB0(t+2)   p2: stage UA0(t+2)   p3: stage UB1(t+2)
// Every phase ends with vmcnt(10) (5 units in flight): it retires the unit the next phase reads
// (B0(t+1) before p3, A0(t+1) before p0 of t+1, B1 before p1, A1 before p2).
template <bool STAMP>
__global__ __launch_bounds__(512) void t8b_kernel(const Args p) {
  constexpr int ROWB = 128, UNIT = 128 * ROWB, STAGE = 4 * UNIT;
  constexpr int UA0 = 0, UA1 = UNIT, UB0 = 2 * UNIT, UB1 = 3 * UNIT;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int wg = xcd_remap((int)blockIdx.x, ntiles);
  const int64_t m0 = (int64_t)(wg / tiles_n) * 256, n0 = (int64_t)(wg % tiles_n) * 256;
  const int nk = p.K / 64;

  const int drow = lane >> 3, dpc = lane & 7;
  const char* sA[2][2];
  const char* sB[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ur = wave * 16 + i * 8 + drow;
    const int ch = (dpc ^ ((ur >> 1) & 7)) * 16;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int lr = (ur >> 6) * 128 + q * 64 + (ur & 63);
      sA[q][i] = (const char*)p.a + (m0 + lr) * p.lda * 2 + ch;
      const int lc = (ur >> 5) * 64 + q * 32 + t8_perm(ur & 31);
      sB[q][i] = (const char*)p.b + (n0 + lc) * p.ldb * 2 + ch;
    }
  }
  auto stage = [&](const char* const* src, int unit_off, int kt, int buf) __attribute__((always_inline)) {
    kt = kt < nk ? kt : nk - 1;
    char* dst = smem + buf * STAGE + unit_off + wave * 16 * ROWB;
    glds16(src[0] + (int64_t)kt * ROWB, dst);
    glds16(src[1] + (int64_t)kt * ROWB, dst + 8 * ROWB);
  };
  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;
  const int c0 = ((0 + fq) ^ sw) * 16, c1 = ((4 + fq) ^ sw) * 16;
  const int aoff = (wr * 64 + frow) * ROWB, boff = (wc * 32 + frow) * ROWB;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x4 aR[4][2], b0R[2][2], b1R[2][2], bN[2][2];
  auto loadA = [&](const char* base, int mq) __attribute__((always_inline)) {
    const char* r = base + (mq ? UA1 : UA0) + aoff;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      aR[f][0] = *(const i32x4*)(r + f * 16 * ROWB + c0);
      aR[f][1] = *(const i32x4*)(r + f * 16 * ROWB + c1);
    }
  };
  auto loadB = [&](const char* base, int nq, i32x4 (&dst)[2][2]) __attribute__((always_inline)) {
    const char* r = base + (nq ? UB1 : UB0) + boff;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      dst[g][0] = *(const i32x4*)(r + g * 16 * ROWB + c0);
      dst[g][1] = *(const i32x4*)(r + g * 16 * ROWB + c1);
    }
  };
  auto comp = [&](int mq, int nq, const i32x4 (&bR)[2][2]) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g)
          acc[mq * 4 + f][nq * 2 + g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, bR[g][kk]), __builtin_bit_cast(bf16x8, aR[f][kk]),
              acc[mq * 4 + f][nq * 2 + g], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
#define T8_BAR()                         \
  do {                                   \
    __builtin_amdgcn_sched_barrier(0);   \
    __builtin_amdgcn_s_barrier();        \
    __builtin_amdgcn_sched_barrier(0);   \
  } while (0)
  const bool g1 = wr == 1;  // wave-uniform
  // prologue: issue order UB0(0) UA0(0) UB1(0) UA1(0) UB0(1) UA0(1) UB1(1); vmcnt(10) retires
  // the first two; B0(0) -> registers (retired before any barrier: its unit is restaged in p1)
  stage(sB[0], UB0, 0, 0);
  stage(sA[0], UA0, 0, 0);
  stage(sB[1], UB1, 0, 0);
  stage(sA[1], UA1, 0, 0);
  stage(sB[0], UB0, 1, 1);
  stage(sA[0], UA0, 1, 1);
  stage(sB[1], UB1, 1, 1);
  wait_vm<10>();
  T8_BAR();
  loadB(smem, 0, b0R);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (g1) T8_BAR();
  // the loop body is written twice (even / odd K-tile) so the B0 register sets swap statically
  auto ktile = [&](int t, i32x4 (&bc)[2][2], i32x4 (&bn)[2][2]) __attribute__((always_inline)) {
    const int b = t & 1, nb = b ^ 1;
    const char* cur = smem + b * STAGE;
    loadA(cur, 0);  // p0: A0(t)
    stage(sA[1], UA1, t + 1, nb);
    if (g1) wait_vm<10>();
    T8_BAR();
    comp(0, 0, bc);
    if (!g1) wait_vm<10>();
    T8_BAR();
    loadB(cur, 1, b1R);  // p1: B1(t)
    stage(sB[0], UB0, t + 2, b);
    if (g1) wait_vm<10>();
    T8_BAR();
    comp(0, 1, b1R);
    if (!g1) wait_vm<10>();
    T8_BAR();
    loadA(cur, 1);  // p2: A1(t)
    stage(sA[0], UA0, t + 2, b);
    if (g1) wait_vm<10>();
    T8_BAR();
    comp(1, 1, b1R);
    if (!g1) wait_vm<10>();
    T8_BAR();
    loadB(smem + nb * STAGE, 0, bn);  // p3: B0(t+1) -> next set
    stage(sB[1], UB1, t + 2, b);
    if (g1) wait_vm<10>();
    T8_BAR();
    comp(1, 0, bc);
    if (!g1) wait_vm<10>();
    T8_BAR();
  };
  int t = 0;
  for (; t + 1 < nk; t += 2) {
    ktile(t, b0R, bN);
    ktile(t + 1, bN, b0R);
  }
  if (t < nk) ktile(t, b0R, bN);
  if (!g1) T8_BAR();
#undef T8_BAR
  wait_vm<0>();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    char* crow = (char*)p.c + (m0 + wr * 128 + (i >> 2) * 64 + (i & 3) * 16 + frow) * p.ldc * 2;
#pragma unroll
    for (int nq = 0; nq < 2; ++nq) {
      const f32x4 v0 = acc[i][nq * 2], v1 = acc[i][nq * 2 + 1];
      bf16x8 o = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                  (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
      *(uint4*)(crow + (n0 + wc * 64 + nq * 32 + fq * 8) * 2) = __builtin_bit_cast(uint4, o);
    }
  }
}


// t4: the ping-pong with 2 phases per K-tile and 32 MFMAs per compute section (half the barriers
// of t8). Phase A: read A0 + B0 + B1 (16), compute (0,0)+(0,1); phase B: read A1 (8), compute
// (1,1)+(1,0). Intervals per K-tile t: g0 reads I_{4t}, I_{4t+2}; g1 one later. Every read
// section ends with lgkmcnt(0) before its barrier, so a unit is restaged from the interval after
// its last read: phase B of t stages UB0/UB1(t+2), phase A of t+1 stages UA0/UA1(t+2) (buffer t&1).
// RAW: vmcnt(6) after phase B (retires A0 of K-tile t+1, the youngest unit phase A of t+1 reads),
// vmcnt(8) after phase A (retires A1 of the current K-tile).
template <bool STAMP>
__global__ __launch_bounds__(512) void t4_kernel(const Args p) {
  constexpr int ROWB = 128, UNIT = 128 * ROWB, STAGE = 4 * UNIT;
  constexpr int UA0 = 0, UA1 = UNIT, UB0 = 2 * UNIT, UB1 = 3 * UNIT;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int wg = xcd_remap((int)blockIdx.x, ntiles);
  const int64_t m0 = (int64_t)(wg / tiles_n) * 256, n0 = (int64_t)(wg % tiles_n) * 256;
  const int nk = p.K / 64;
  const int drow = lane >> 3, dpc = lane & 7;
  const char* sA[2][2];
  const char* sB[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ur = wave * 16 + i * 8 + drow;
    const int ch = (dpc ^ ((ur >> 1) & 7)) * 16;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int lr = (ur >> 6) * 128 + q * 64 + (ur & 63);
      sA[q][i] = (const char*)p.a + (m0 + lr) * p.lda * 2 + ch;
      const int lc = (ur >> 5) * 64 + q * 32 + t8_perm(ur & 31);
      sB[q][i] = (const char*)p.b + (n0 + lc) * p.ldb * 2 + ch;
    }
  }
  auto stage = [&](const char* const* src, int unit_off, int kt, int buf) __attribute__((always_inline)) {
    kt = kt < nk ? kt : nk - 1;
    char* dst = smem + buf * STAGE + unit_off + wave * 16 * ROWB;
    glds16(src[0] + (int64_t)kt * ROWB, dst);
    glds16(src[1] + (int64_t)kt * ROWB, dst + 8 * ROWB);
  };
  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;
  const int c0 = ((0 + fq) ^ sw) * 16, c1 = ((4 + fq) ^ sw) * 16;
  const int aoff = (wr * 64 + frow) * ROWB, boff = (wc * 32 + frow) * ROWB;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x4 aR[4][2], b0R[2][2], b1R[2][2];
  auto loadA = [&](const char* base, int mq) __attribute__((always_inline)) {
    const char* r = base + (mq ? UA1 : UA0) + aoff;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      aR[f][0] = *(const i32x4*)(r + f * 16 * ROWB + c0);
      aR[f][1] = *(const i32x4*)(r + f * 16 * ROWB + c1);
    }
  };
  auto loadB = [&](const char* base, int nq, i32x4 (&dst)[2][2]) __attribute__((always_inline)) {
    const char* r = base + (nq ? UB1 : UB0) + boff;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      dst[g][0] = *(const i32x4*)(r + g * 16 * ROWB + c0);
      dst[g][1] = *(const i32x4*)(r + g * 16 * ROWB + c1);
    }
  };
  auto mm = [&](int mq, int nq, const i32x4 (&bR)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g)
          acc[mq * 4 + f][nq * 2 + g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, bR[g][kk]), __builtin_bit_cast(bf16x8, aR[f][kk]),
              acc[mq * 4 + f][nq * 2 + g], 0, 0, 0);
  };
#define T4_BAR()                         \
  do {                                   \
    __builtin_amdgcn_sched_barrier(0);   \
    __builtin_amdgcn_s_barrier();        \
    __builtin_amdgcn_sched_barrier(0);   \
  } while (0)
#define T4_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
  const bool g1 = wr == 1;
  // prologue = the steady-state issue order up to "end of phase B of K-tile -1":
  // B0 B1 A0 A1 of K-tile 0, B0 B1 of K-tile 1; vmcnt(6) retires B0, B1, A0 of K-tile 0
  stage(sB[0], UB0, 0, 0);
  stage(sB[1], UB1, 0, 0);
  stage(sA[0], UA0, 0, 0);
  stage(sA[1], UA1, 0, 0);
  stage(sB[0], UB0, 1, 1);
  stage(sB[1], UB1, 1, 1);
  wait_vm<6>();
  T4_BAR();
  if (g1) T4_BAR();
  for (int t = 0; t < nk; ++t) {
    const int b = t & 1;
    const char* cur = smem + b * STAGE;
    // phase A: read A0 + B0 + B1 of t; stage UA0/UA1(t+1) into the other buffer
    loadB(cur, 0, b0R);
    loadB(cur, 1, b1R);
    loadA(cur, 0);
    stage(sA[0], UA0, t + 1, b ^ 1);
    stage(sA[1], UA1, t + 1, b ^ 1);
    T4_LGKM0();
    if (g1) wait_vm<8>();  // retires A1 of K-tile t (younger: B0/B1(t+1), A0/A1(t+1))
    T4_BAR();
    __builtin_amdgcn_s_setprio(1);
    mm(0, 0, b0R);
    mm(0, 1, b1R);
    __builtin_amdgcn_s_setprio(0);
    if (!g1) wait_vm<8>();
    T4_BAR();
    // phase B: A1; stage B0/B1 of K-tile t+2 into this buffer (its B units were read in phase A)
    loadA(cur, 1);
    stage(sB[0], UB0, t + 2, b);
    stage(sB[1], UB1, t + 2, b);
    T4_LGKM0();
    if (g1) wait_vm<6>();  // retires A0 of K-tile t+1 (younger: A1(t+1), B0/B1(t+2))
    T4_BAR();
    __builtin_amdgcn_s_setprio(1);
    mm(1, 1, b1R);
    mm(1, 0, b0R);
    __builtin_amdgcn_s_setprio(0);
    if (!g1) wait_vm<6>();
    T4_BAR();
  }
  if (!g1) T4_BAR();
#undef T4_BAR
#undef T4_LGKM0
  wait_vm<0>();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    char* crow = (char*)p.c + (m0 + wr * 128 + (i >> 2) * 64 + (i & 3) * 16 + frow) * p.ldc * 2;
#pragma unroll
    for (int nq = 0; nq < 2; ++nq) {
      const f32x4 v0 = acc[i][nq * 2], v1 = acc[i][nq * 2 + 1];
      bf16x8 o = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                  (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
      *(uint4*)(crow + (n0 + wc * 64 + nq * 32 + fq * 8) * 2) = __builtin_bit_cast(uint4, o);
    }
  }
}


// pt4: persistent t4 (tiles streamed back to back like pt8). A tile's quadrants are stored right
// after their last MFMAs: Q00 + Q01 after phase A of its last K-tile, Q11 + Q10 after phase B.
// vmcnt counts (NS = C stores per quadrant per wave), per K-tile kind:
//   normal:            A end 8, B end 6
//   LAST of a tile:    A end g0 8+2NS / g1 8,   B end g0 6+4NS / g1 6+2NS
//   FIRST after LAST:  A end 8+4NS (both),      B end 6
template <bool STAMP, int SKIP = 0>  // SKIP (timing ablations): 1 no LDS-DMA after the first 2 K-tiles, 2 no C stores, 4 no MFMA, 8 no LDS reads
__global__ __launch_bounds__(512) void pt4_kernel(const Args p) {
  constexpr int ROWB = 128, UNIT = 128 * ROWB, STAGE = 4 * UNIT;
  constexpr int UA0 = 0, UA1 = UNIT, UB0 = 2 * UNIT, UB1 = 3 * UNIT;
  constexpr int NS = 4;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int nk = p.K / 64;
  const int my_tiles =
      ((int)blockIdx.x < ntiles) ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  if (my_tiles == 0) return;
  // stagger experiments (round 2): delay some blocks at the start so the chip-wide C-store
  // bursts at tile ends are spread in time. 64: odd blocks ~half a tile; 128: odd blocks ~a
  // sixth; 192: block % 4 phases of ~a quarter tile each
  if constexpr ((SKIP & 192) == 64) {
    if (blockIdx.x & 1) for (int i = 0; i < 3; ++i) __builtin_amdgcn_s_sleep(127);
  } else if constexpr ((SKIP & 192) == 128) {
    if (blockIdx.x & 1) __builtin_amdgcn_s_sleep(127);
  } else if constexpr ((SKIP & 192) == 192) {
    for (int i = 0; i < (int)(blockIdx.x & 3) * 2; ++i) __builtin_amdgcn_s_sleep(100);
  }
  // LDS-DMA sources: per-lane 32-bit byte offsets inside a tile's A / B panels (row * ld + swizzled
  // chunk) plus wave-uniform panel bases, so the per-tile state is two scalar pointers
  const int drow = lane >> 3, dpc = lane & 7;
  unsigned offA[2][2], offB[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ur = wave * 16 + i * 8 + drow;
    const int ch = (dpc ^ ((ur >> 1) & 7)) * 16;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int lr = (ur >> 6) * 128 + q * 64 + (ur & 63);
      offA[q][i] = (unsigned)(lr * p.lda * 2 + ch);
      const int lc = (ur >> 5) * 64 + q * 32 + t8_perm(ur & 31);
      offB[q][i] = (unsigned)(lc * p.ldb * 2 + ch);
    }
  }
  const char* baseA = nullptr;
  const char* baseB = nullptr;
  int src_tile = -1;
  auto origin = [&](int ti, int64_t& m0, int64_t& n0) __attribute__((always_inline)) {
    const int wg = xcd_remap((int)blockIdx.x + ti * (int)gridDim.x, ntiles);
    m0 = (int64_t)(wg / tiles_n) * 256;
    n0 = (int64_t)(wg % tiles_n) * 256;
  };
  struct Cur { int ti, kt; };
  auto adv = [&](Cur& c) __attribute__((always_inline)) {
    if (c.ti == my_tiles - 1 && c.kt == nk - 1) return;
    if (++c.kt == nk) { c.kt = 0; ++c.ti; }
  };
  auto stage = [&](int which, int unit_off, Cur c, int buf) __attribute__((always_inline)) {
    if constexpr ((SKIP & 1) != 0) {
      if (c.ti > 0 || c.kt >= 2) return;
    }
    if (c.ti != src_tile) {
      int64_t m0, n0;
      origin(c.ti, m0, n0);
      baseA = (const char*)p.a + m0 * p.lda * 2;
      baseB = (const char*)p.b + n0 * p.ldb * 2;
      src_tile = c.ti;
    }
    const char* base = (which < 2 ? baseA : baseB) + (int64_t)c.kt * ROWB;
    const unsigned* off = which < 2 ? offA[which] : offB[which - 2];
    char* dst = smem + buf * STAGE + unit_off + wave * 16 * ROWB;
    if constexpr ((SKIP & 8192) != 0) {
      // buffer form: wave-uniform descriptor of the tile panel, the per-lane 32-bit offset as
      // voffset and the K-tile offset as soffset: no per-lane 64-bit address arithmetic
      const uint64_t u = (uint64_t)(which < 2 ? baseA : baseB);
      const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
      const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(((uint64_t)hi << 32) | lo), 0, 0x7FFFFFF0, 0x00020000);
      const int soff = __builtin_amdgcn_readfirstlane(c.kt * ROWB);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)dst, 16, off[0], soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)(dst + 8 * ROWB), 16, off[1], soff,
                                               0, 0);
    } else {
      glds16(base + off[0], dst);
      glds16(base + off[1], dst + 8 * ROWB);
    }
  };
  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;
  const int c0 = ((0 + fq) ^ sw) * 16, c1 = ((4 + fq) ^ sw) * 16;
  const int aoff = (wr * 64 + frow) * ROWB, boff = (wc * 32 + frow) * ROWB;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x4 aR[4][2], bR[2][2][2];
  auto loadA = [&](const char* base, int mq) __attribute__((always_inline)) {
    if constexpr ((SKIP & 8) != 0) return;
    const char* r = base + (mq ? UA1 : UA0) + aoff;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      aR[f][0] = *(const i32x4*)(r + f * 16 * ROWB + c0);
      aR[f][1] = *(const i32x4*)(r + f * 16 * ROWB + c1);
    }
  };
  auto loadB = [&](const char* base, int nq) __attribute__((always_inline)) {
    if constexpr ((SKIP & 8) != 0) return;
    const char* r = base + (nq ? UB1 : UB0) + boff;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      bR[nq][g][0] = *(const i32x4*)(r + g * 16 * ROWB + c0);
      bR[nq][g][1] = *(const i32x4*)(r + g * 16 * ROWB + c1);
    }
  };
  auto mm = [&](int mq, int nq) __attribute__((always_inline)) {
    if constexpr ((SKIP & 4) != 0) {
#pragma unroll
      for (int f = 0; f < 4; ++f) asm volatile("" ::"v"(aR[f][0]), "v"(bR[nq][0][1]));
      return;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g)
          acc[mq * 4 + f][nq * 2 + g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, bR[nq][g][kk]), __builtin_bit_cast(bf16x8, aR[f][kk]),
              acc[mq * 4 + f][nq * 2 + g], 0, 0, 0);
  };
  int ti = 0;
  // one fragment row-block (f) of quadrant (mq, nq) of tile sti: 8 bf16 per lane, then zeroed
  auto store_frag = [&](int mq, int nq, int f, int sti) __attribute__((always_inline)) {
    const int i = mq * 4 + f;
    if constexpr ((SKIP & 2) != 0) {
      asm volatile("" ::"v"(acc[i][nq * 2]), "v"(acc[i][nq * 2 + 1]));
      return;
    }
    int64_t m0, n0;
    origin(sti, m0, n0);
    if constexpr ((SKIP & 512) != 0) {  // timing only: every tile of a block stores to one small
      m0 = (int64_t)(blockIdx.x % 64) * 256;  // C region (L2-resident lines, no HBM write stream)
      n0 = 0;
    }
    char* crow = (char*)p.c + (m0 + wr * 128 + mq * 64 + f * 16 + frow) * p.ldc * 2;
    const f32x4 v0 = acc[i][nq * 2], v1 = acc[i][nq * 2 + 1];
    bf16x8 o = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
    if constexpr ((SKIP & (16384 | 32768)) != 0) {
      // C through a buffer descriptor with explicit cache bits: 16384 = sc1 (write-through, the
      // line leaves this XCD's L2), + 16 = sc1 | nt, 32768 = sc0 | sc1
      constexpr int AUX = (SKIP & 32768) ? 17 : ((SKIP & 16) ? 18 : 16);
      const __amdgpu_buffer_rsrc_t rc =
          __builtin_amdgcn_make_buffer_rsrc((void*)p.c, 0, 0x7FFFFFF0, 0x00020000);
      const int64_t off = (crow - (char*)p.c) + (n0 + wc * 64 + nq * 32 + fq * 8) * 2;
      typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), rc, (unsigned)off, 0,
                                             AUX);
    } else if constexpr ((SKIP & 32) != 0) {  // timing only: same bytes, one full 128 B line per 8 lanes
      const int rl = lane >> 3, ch = lane & 7;
      char* rrow = (char*)p.c + (m0 + wr * 128 + mq * 64 + f * 16 + nq * 8 + rl) * p.ldc * 2;
      char* dst = rrow + (n0 + wc * 64 + ch * 8) * 2;
      if constexpr ((SKIP & 16) != 0) __builtin_nontemporal_store(__builtin_bit_cast(i32x4, o), (i32x4*)dst);
      else *(uint4*)dst = __builtin_bit_cast(uint4, o);
    } else if constexpr ((SKIP & 16) != 0) {  // non-temporal (streaming) store: C is never re-read
      __builtin_nontemporal_store(__builtin_bit_cast(i32x4, o),
                                  (i32x4*)(crow + (n0 + wc * 64 + nq * 32 + fq * 8) * 2));
    } else {
      *(uint4*)(crow + (n0 + wc * 64 + nq * 32 + fq * 8) * 2) = __builtin_bit_cast(uint4, o);
    }
    acc[i][nq * 2] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc[i][nq * 2 + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto store_q = [&](int mq, int nq, int sti) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int f = 0; f < 4; ++f) store_frag(mq, nq, f, sti);
    __builtin_amdgcn_sched_barrier(0);
  };
  // MFMAs of quadrants (mq, na) then (mq, nb) — 32 — with the 8 fragment stores of quadrants
  // (smq, 0) and (smq, 1) of tile sti interleaved, one after every 4 MFMAs (SKIP & 256): spreads
  // the C-store issue over a compute section instead of bunching it after one
  auto mm_st = [&](int mq, int na, int nb, int smq, int sti) __attribute__((always_inline)) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int nq = half ? nb : na;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if constexpr ((SKIP & 1024) == 0) __builtin_amdgcn_sched_barrier(0);
        const int kk = c >> 1;
#pragma unroll
        for (int ff = 0; ff < 2; ++ff)
#pragma unroll
          for (int g = 0; g < 2; ++g) {
            const int f = (c & 1) * 2 + ff;
            acc[mq * 4 + f][nq * 2 + g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, bR[nq][g][kk]), __builtin_bit_cast(bf16x8, aR[f][kk]),
                acc[mq * 4 + f][nq * 2 + g], 0, 0, 0);
          }
        const int si = half * 4 + c;  // store #si: quadrant (smq, si >> 2), fragment si & 3
        store_frag(smq, si >> 2, si & 3, sti);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
#define T4_BAR()                         \
  do {                                   \
    __builtin_amdgcn_sched_barrier(0);   \
    __builtin_amdgcn_s_barrier();        \
    __builtin_amdgcn_sched_barrier(0);   \
  } while (0)
#define T4_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
  const bool g1 = wr == 1;
  // STAMP: per-wave cycle buckets (s_memtime, scalar): 0 LDS-read phase up to lgkmcnt(0), 1 vmcnt
  // waits, 2 barriers, 3 MFMA issue, 4 C stores, 5 whole stream
  unsigned long long st[16] = {}, tprev = 0;
  auto T = [&](int bucket) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
      if (bucket >= 0) st[bucket] += t - tprev;
      tprev = t;
    }
  };
  // stage cursors: qa = K-tile h+1 (A units staged in phase A), qb = h+2 (B units in phase B)
  Cur q0{0, 0}, q1{0, 0};
  adv(q1);
  stage(2, UB0, q0, 0);
  stage(3, UB1, q0, 0);
  stage(0, UA0, q0, 0);
  stage(1, UA1, q0, 0);
  stage(2, UB0, q1, 1);
  stage(3, UB1, q1, 1);
  Cur qa = q1, qb = q1;
  adv(qb);
  wait_vm<6>();
  T4_BAR();
  if (g1) T4_BAR();
  T(-1);
  const unsigned long long t_start = tprev;
  // KIND: 0 normal, 1 last K-tile of a tile, 2 first K-tile after a tile's last, 3 second
  // (3 only with interleaved stores, SKIP & 256: Q00/Q01 of the finished tile are stored inside
  // phase B of its last K-tile, Q11/Q10 inside phase A of the next tile's first K-tile; the
  // counted waits keep exactly the ops younger than the unit a phase reads in flight)
  constexpr bool ILS = (SKIP & 256) != 0;
  auto iter = [&](int h, auto kind_tag) __attribute__((always_inline)) {
    constexpr int KIND = decltype(kind_tag)::value;
    const int b = h & 1;
    const char* cur = smem + b * STAGE;
    // SKIP & 65536 (timing only, wrong results): balanced reads, phase A B0 + A0, phase B B1 + A1
    loadB(cur, 0);  // phase A
    if constexpr ((SKIP & 65536) == 0) loadB(cur, 1);
    loadA(cur, 0);
    T(0);
    stage(0, UA0, qa, b ^ 1);
    stage(1, UA1, qa, b ^ 1);
    T(1);
    T4_LGKM0();
    T(2);
    if constexpr (ILS) {
      if (g1) wait_vm<KIND == 2 || KIND == 3 ? 8 + 2 * NS : 8>();
    } else {
      if (g1) wait_vm<KIND == 2 ? 8 + 4 * NS : 8>();
    }
    T(6);
    T4_BAR();
    T(7);
    if constexpr ((SKIP & 2048) == 0) __builtin_amdgcn_s_setprio((SKIP & 4096) ? 0 : 1);
    if constexpr (ILS && KIND == 2) {
      mm_st(0, 0, 1, 1, ti - 1);
    } else {
      mm(0, 0);
      mm(0, 1);
    }
    if constexpr ((SKIP & 2048) == 0) __builtin_amdgcn_s_setprio((SKIP & 4096) ? 1 : 0);
    T(11);
    if constexpr (!ILS && KIND == 1) { store_q(0, 0, ti); store_q(0, 1, ti); }
    T(13);
    if constexpr (ILS) {
      if (!g1) wait_vm<KIND == 2 ? 8 + 4 * NS : (KIND == 3 ? 8 + 2 * NS : 8)>();
    } else {
      if (!g1) wait_vm<KIND == 1 ? 8 + 2 * NS : (KIND == 2 ? 8 + 4 * NS : 8)>();
    }
    T(6);
    T4_BAR();
    T(8);
    loadA(cur, 1);  // phase B
    if constexpr ((SKIP & 65536) != 0) loadB(cur, 1);
    T(3);
    stage(2, UB0, qb, b);
    stage(3, UB1, qb, b);
    T(4);
    T4_LGKM0();
    T(5);
    if constexpr (ILS) {
      if (g1) wait_vm<KIND == 2 ? 6 + 2 * NS : 6>();
    } else {
      if (g1) wait_vm<KIND == 1 ? 6 + 2 * NS : 6>();
    }
    T(6);
    T4_BAR();
    T(9);
    if constexpr ((SKIP & 2048) == 0) __builtin_amdgcn_s_setprio((SKIP & 4096) ? 0 : 1);
    if constexpr (ILS && KIND == 1) {
      mm_st(1, 1, 0, 0, ti);
    } else {
      mm(1, 1);
      mm(1, 0);
    }
    if constexpr ((SKIP & 2048) == 0) __builtin_amdgcn_s_setprio((SKIP & 4096) ? 1 : 0);
    T(12);
    if constexpr (!ILS && KIND == 1) { store_q(1, 1, ti); store_q(1, 0, ti); }
    T(13);
    if constexpr (ILS) {
      if (!g1) wait_vm<KIND == 1 || KIND == 2 ? 6 + 2 * NS : 6>();
    } else {
      if (!g1) wait_vm<KIND == 1 ? 6 + 4 * NS : 6>();
    }
    T(6);
    T4_BAR();
    T(10);
    qa = qb;
    adv(qb);
  };
  int h = 0;
  for (ti = 0; ti < my_tiles; ++ti) {
    int t = 0;
    if (ti > 0) { iter(h, std::integral_constant<int, 2>{}); ++h; ++t; }
    if (ILS && ti > 0) { iter(h, std::integral_constant<int, 3>{}); ++h; ++t; }
    for (; t < nk - 1; ++t, ++h) iter(h, std::integral_constant<int, 0>{});
    iter(h, std::integral_constant<int, 1>{});
    ++h;
  }
  if constexpr (ILS) {  // the last tile's Q11 / Q10 have no next tile to hide under
    store_q(1, 1, my_tiles - 1);
    store_q(1, 0, my_tiles - 1);
  }
  if (!g1) T4_BAR();
#undef T4_BAR
#undef T4_LGKM0
  wait_vm<0>();
  if constexpr (STAMP) {
    T(-1);
    st[14] = tprev - t_start;
    if (lane == 0) {
      unsigned long long* o = p.stamps + ((size_t)blockIdx.x * 8 + wave) * 16;
#pragma unroll
      for (int j = 0; j < 15; ++j) o[j] = st[j];
      o[15] = (unsigned long long)my_tiles;
    }
  }
}


template <bool STAMP, int SKIP = 0>  // SKIP (timing ablations): 1 no LDS-DMA after the first 2 K-tiles, 2 no C stores, 4 no MFMA, 8 no LDS reads
__global__ __launch_bounds__(512) void pt4b_kernel(const Args p) {
  constexpr int ROWB = 128, UNIT = 128 * ROWB, STAGE = 4 * UNIT;
  constexpr int UA0 = 0, UA1 = UNIT, UB0 = 2 * UNIT, UB1 = 3 * UNIT;
  constexpr int NS = 4;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int nk = p.K / 64;
  const int my_tiles =
      ((int)blockIdx.x < ntiles) ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  if (my_tiles == 0) return;
  // LDS-DMA sources: per-lane 32-bit byte offsets inside a tile's A / B panels (row * ld + swizzled
  // chunk) plus wave-uniform panel bases, so the per-tile state is two scalar pointers
  const int drow = lane >> 3, dpc = lane & 7;
  unsigned offA[2][2], offB[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ur = wave * 16 + i * 8 + drow;
    const int ch = (dpc ^ ((ur >> 1) & 7)) * 16;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int lr = (ur >> 6) * 128 + q * 64 + (ur & 63);
      offA[q][i] = (unsigned)(lr * p.lda * 2 + ch);
      const int lc = (ur >> 5) * 64 + q * 32 + t8_perm(ur & 31);
      offB[q][i] = (unsigned)(lc * p.ldb * 2 + ch);
    }
  }
  const char* baseA = nullptr;
  const char* baseB = nullptr;
  int src_tile = -1;
  auto origin = [&](int ti, int64_t& m0, int64_t& n0) __attribute__((always_inline)) {
    const int wg = xcd_remap((int)blockIdx.x + ti * (int)gridDim.x, ntiles);
    m0 = (int64_t)(wg / tiles_n) * 256;
    n0 = (int64_t)(wg % tiles_n) * 256;
  };
  struct Cur { int ti, kt; };
  auto adv = [&](Cur& c) __attribute__((always_inline)) {
    if (c.ti == my_tiles - 1 && c.kt == nk - 1) return;
    if (++c.kt == nk) { c.kt = 0; ++c.ti; }
  };
  auto stage = [&](int which, int unit_off, Cur c, int buf) __attribute__((always_inline)) {
    if constexpr ((SKIP & 1) != 0) {
      if (c.ti > 0 || c.kt >= 2) return;
    }
    if (c.ti != src_tile) {
      int64_t m0, n0;
      origin(c.ti, m0, n0);
      baseA = (const char*)p.a + m0 * p.lda * 2;
      baseB = (const char*)p.b + n0 * p.ldb * 2;
      src_tile = c.ti;
    }
    const char* base = (which < 2 ? baseA : baseB) + (int64_t)c.kt * ROWB;
    const unsigned* off = which < 2 ? offA[which] : offB[which - 2];
    char* dst = smem + buf * STAGE + unit_off + wave * 16 * ROWB;
    glds16(base + off[0], dst);
    glds16(base + off[1], dst + 8 * ROWB);
  };
  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;
  const int c0 = ((0 + fq) ^ sw) * 16, c1 = ((4 + fq) ^ sw) * 16;
  const int aoff = (wr * 64 + frow) * ROWB, boff = (wc * 32 + frow) * ROWB;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x4 aR[4][2], bR[2][2][2];
  auto loadA = [&](const char* base, int mq) __attribute__((always_inline)) {
    const char* r = base + (mq ? UA1 : UA0) + aoff;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      aR[f][0] = *(const i32x4*)(r + f * 16 * ROWB + c0);
      aR[f][1] = *(const i32x4*)(r + f * 16 * ROWB + c1);
    }
  };
  auto loadB = [&](const char* base, int nq) __attribute__((always_inline)) {
    const char* r = base + (nq ? UB1 : UB0) + boff;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      bR[nq][g][0] = *(const i32x4*)(r + g * 16 * ROWB + c0);
      bR[nq][g][1] = *(const i32x4*)(r + g * 16 * ROWB + c1);
    }
  };
  auto mm = [&](int mq, int nq) __attribute__((always_inline)) {
    if constexpr ((SKIP & 4) != 0) {
#pragma unroll
      for (int f = 0; f < 4; ++f) asm volatile("" ::"v"(aR[f][0]), "v"(bR[nq][0][1]));
      return;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g)
          acc[mq * 4 + f][nq * 2 + g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, bR[nq][g][kk]), __builtin_bit_cast(bf16x8, aR[f][kk]),
              acc[mq * 4 + f][nq * 2 + g], 0, 0, 0);
  };
  int ti = 0;
  auto store_q = [&](int mq, int nq) __attribute__((always_inline)) {
    int64_t m0, n0;
    origin(ti, m0, n0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int i = mq * 4 + f;
      char* crow = (char*)p.c + (m0 + wr * 128 + mq * 64 + f * 16 + frow) * p.ldc * 2;
      const f32x4 v0 = acc[i][nq * 2], v1 = acc[i][nq * 2 + 1];
      bf16x8 o = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                  (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
      *(uint4*)(crow + (n0 + wc * 64 + nq * 32 + fq * 8) * 2) = __builtin_bit_cast(uint4, o);
      acc[i][nq * 2] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc[i][nq * 2 + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __builtin_amdgcn_sched_barrier(0);
  };
#define T4_BAR()                         \
  do {                                   \
    __builtin_amdgcn_sched_barrier(0);   \
    __builtin_amdgcn_s_barrier();        \
    __builtin_amdgcn_sched_barrier(0);   \
  } while (0)
#define T4_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
  const bool g1 = wr == 1;
  // every unit restaged right after its last read: phase A of h stages A1(h+1) (A1(h-1) was
  // read in phase B of h-1), phase B of h stages A0 / B0 / B1 of h+2 (read in phase A of h).
  // Cursors: qa = h+1, qb = h+2. Prologue = the steady-state issue order up to the end of phase B
  // of K-tile -1: A0 B0 B1 (0), A1 (0), A0 B0 B1 (1); 8 younger than B1(0).
  Cur q0{0, 0}, q1{0, 0};
  adv(q1);
  stage(0, UA0, q0, 0);
  stage(2, UB0, q0, 0);
  stage(3, UB1, q0, 0);
  stage(1, UA1, q0, 0);
  stage(0, UA0, q1, 1);
  stage(2, UB0, q1, 1);
  stage(3, UB1, q1, 1);
  Cur qa = q1, qb = q1;
  adv(qb);
  wait_vm<8>();
  T4_BAR();
  if (g1) T4_BAR();
  // KIND: 0 normal, 1 last K-tile of a tile, 2 first K-tile after a tile's last
  auto iter = [&](int h, auto kind_tag) __attribute__((always_inline)) {
    constexpr int KIND = decltype(kind_tag)::value;
    const int b = h & 1;
    const char* cur = smem + b * STAGE;
    loadB(cur, 0);  // phase A
    loadB(cur, 1);
    loadA(cur, 0);
    stage(1, UA1, qa, b ^ 1);
    T4_LGKM0();
    if (g1) wait_vm<KIND == 2 ? 8 + 4 * NS : 8>();
    T4_BAR();
    __builtin_amdgcn_s_setprio(1);
    mm(0, 0);
    mm(0, 1);
    __builtin_amdgcn_s_setprio(0);
    if constexpr (KIND == 1) { store_q(0, 0); store_q(0, 1); }
    if (!g1) wait_vm<KIND == 1 ? 8 + 2 * NS : (KIND == 2 ? 8 + 4 * NS : 8)>();
    T4_BAR();
    loadA(cur, 1);  // phase B
    stage(0, UA0, qb, b);
    stage(2, UB0, qb, b);
    stage(3, UB1, qb, b);
    T4_LGKM0();
    if (g1) wait_vm<KIND == 0 ? 8 : 8 + 2 * NS>();
    T4_BAR();
    __builtin_amdgcn_s_setprio(1);
    mm(1, 1);
    mm(1, 0);
    __builtin_amdgcn_s_setprio(0);
    if constexpr (KIND == 1) { store_q(1, 1); store_q(1, 0); }
    if (!g1) wait_vm<KIND == 1 ? 8 + 4 * NS : (KIND == 2 ? 8 + 2 * NS : 8)>();
    T4_BAR();
    qa = qb;
    adv(qb);
  };
  int h = 0;
  for (ti = 0; ti < my_tiles; ++ti) {
    int t = 0;
    if (ti > 0) { iter(h, std::integral_constant<int, 2>{}); ++h; ++t; }
    for (; t < nk - 1; ++t, ++h) iter(h, std::integral_constant<int, 0>{});
    iter(h, std::integral_constant<int, 1>{});
    ++h;
  }
  if (!g1) T4_BAR();
#undef T4_BAR
#undef T4_LGKM0
  wait_vm<0>();
}



// q4: one wave per SIMD. 256x256 tile, 4 waves (2x2) of 128x128, accumulators (256 per lane) in
// AGPRs, fragments double-buffered in VGPRs. Same 16 KB units / swizzle / B permutation as t8
// (UA0 = A rows {0-63,128-191}, UB0 = B cols {0-63,128-191} permuted per 32). A K-tile is 4
// sections of 32 MFMAs (one 64x64 quadrant each); each section reads one fragment set (8
// ds_read_b128) for the next section, snake order by K-tile parity so a set is loaded into
// registers whose last reader has finished:
//   even h: Q00 (ld B1 h) Q01 (ld A1 h) | Q11 (ld A0 h+1) Q10 (ld B1 h+1)
//   odd  h: Q01 (ld B0 h) Q00 (ld A1 h) | Q10 (ld A0 h+1) Q11 (ld B0 h+1)
// "|" = the one barrier per K-tile: K-tile h+1 landed (vmcnt 0) and every read of K-tile h done,
// so the LDS-DMA of K-tile h+2 into h's buffer is issued right after it (S3 + S4).
template <int SCHED, int SKIP = 0>  // SKIP (timing ablations, wrong results): 1 no loop DMA,
__global__ __launch_bounds__(256) void q4_kernel(const Args p) {  // 2 no loop barrier, 4 no MFMA
  constexpr int ROWB = 128, UNIT = 128 * ROWB, STAGE = 4 * UNIT;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int wg = xcd_remap((int)blockIdx.x, ntiles);
  const int64_t m0 = (int64_t)(wg / tiles_n) * 256, n0 = (int64_t)(wg % tiles_n) * 256;
  const int nk = p.K / 64;
  // LDS-DMA: wave stages unit rows [32w, 32w+32) of each unit, 4 x 1 KB instructions per unit.
  // Sources = wave-uniform row bases + one of two per-lane 32-bit offsets (the swizzle repeats
  // every 16 rows, so instructions i and i+2 share a lane pattern).
  const int drow = lane >> 3, dpc = lane & 7;
  int offA[2], offB[4];  // per-lane 32-bit source offsets
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ch = (dpc ^ (((i * 8 + drow) >> 1) & 7)) * 16;
    if (i < 2) offA[i] = (int)(drow * p.lda * 2) + ch;
    offB[i] = (int)(t8_perm(i * 8 + drow) * p.ldb * 2) + ch;
  }
  // wave-uniform bases: A unit row ur = wave*32 + i*8 + drow -> A row (ur>>6)*128 + q*64 + (ur&63)
  const char* baseA = (const char*)p.a + (m0 + (wave >> 1) * 128 + (wave & 1) * 32) * p.lda * 2;
  //                   B unit row -> column (ur>>6)*128 + q*64 + ((ur&63)>>5)*32 + perm(ur&31)
  const char* baseB = (const char*)p.b + (n0 + (wave >> 1) * 128 + (wave & 1) * 32) * p.ldb * 2;
  // SKIP & 8: LDS-DMA through buffer descriptors on the wave's panel bases (row offsets and the
  // K offset in soffset, the fixed per-lane swizzled offsets in voffset: no VALU per piece)
  const __amdgpu_buffer_rsrc_t rqA =
      __builtin_amdgcn_make_buffer_rsrc((void*)baseA, 0, 0x7FFFFFF0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rqB =
      __builtin_amdgcn_make_buffer_rsrc((void*)baseB, 0, 0x7FFFFFF0, 0x00020000);
  auto stage_half = [&](int kt, int buf, int half) __attribute__((always_inline)) {
    if ((SKIP & 1) && kt >= 2) return;
    kt = kt < nk ? kt : nk - 1;  // past the end: K-tile nk-1 again into a buffer no one reads
    char* st = smem + buf * STAGE + wave * 32 * ROWB;
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr ((SKIP & 8) != 0) {
          const unsigned soff = half == 0
              ? (unsigned)((q * 64 + i * 8) * p.lda * 2 + kt * ROWB)
              : (unsigned)((q * 64) * p.ldb * 2 + kt * ROWB);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(half == 0 ? rqA : rqB,
                                                   (LDS_AS void*)(st + (half * 2 + q) * UNIT + i * 8 * ROWB),
                                                   16, (unsigned)(half == 0 ? offA[i & 1] : offB[i]),
                                                   soff, 0, 0);
        } else {
          const char* src = half == 0
              ? baseA + ((int64_t)(q * 64 + i * 8) * p.lda * 2 + (int64_t)kt * ROWB) + offA[i & 1]
              : baseB + ((int64_t)(q * 64) * p.ldb * 2 + (int64_t)kt * ROWB) + offB[i];
          glds16(src, st + (half * 2 + q) * UNIT + i * 8 * ROWB);
        }
      }
  };
  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;
  const int c0 = ((0 + fq) ^ sw) * 16, c1 = ((4 + fq) ^ sw) * 16;
  const int aoff = (wr * 64 + frow) * ROWB, boff = (wc * 64 + frow) * ROWB;
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x4 aR[2][4][2], bR[2][4][2];  // [quadrant][fragment][K-half]
  auto ldA = [&](int kt, int mq) __attribute__((always_inline)) {
    const char* r = smem + (kt & 1) * STAGE + mq * UNIT + aoff;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      aR[mq][f][0] = *(const i32x4*)(r + f * 16 * ROWB + c0);
      aR[mq][f][1] = *(const i32x4*)(r + f * 16 * ROWB + c1);
    }
  };
  auto ldB = [&](int kt, int nq) __attribute__((always_inline)) {
    const char* r = smem + (kt & 1) * STAGE + (2 + nq) * UNIT + boff;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bR[nq][g][0] = *(const i32x4*)(r + g * 16 * ROWB + c0);
      bR[nq][g][1] = *(const i32x4*)(r + g * 16 * ROWB + c1);
    }
  };
  auto mm = [&](int mq, int nq) __attribute__((always_inline)) {
    if constexpr (SKIP & 4) {
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 4; ++g) asm volatile("" :: "v"(aR[mq][f][0]), "v"(bR[nq][g][1]));
      return;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          acc[mq * 4 + f][nq * 4 + g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, bR[nq][g][kk]), __builtin_bit_cast(bf16x8, aR[mq][f][kk]),
              acc[mq * 4 + f][nq * 4 + g], 0, 0, 0);
#pragma unroll
    for (int f = 0; f < 4; ++f)  // keep every accumulator in AGPRs (no loop-carried copies)
#pragma unroll
      for (int g = 0; g < 4; ++g) asm volatile("" : "+a"(acc[mq * 4 + f][nq * 4 + g]));
  };
  // interleave: 1 MFMA then 1 DS read for the first 8 MFMAs (+ VMEM in the DMA sections)
  auto pace = [&](int vmem) __attribute__((always_inline)) {
    if constexpr (SCHED == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        if (vmem) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 24, 0);
    }
  };
// section boundary: the previous section's fragment reads (a whole section of MFMAs old) must
// have landed before this section issues its own, so its MFMAs never wait on the new reads
// (a real S_WAITCNT the compiler's waitcnt pass sees: lgkmcnt(0), vmcnt/expcnt untouched)
#define Q4_SEC()                            \
  do {                                      \
    __builtin_amdgcn_sched_barrier(0);      \
    __builtin_amdgcn_s_waitcnt(0xC07F);     \
    __builtin_amdgcn_sched_barrier(0);      \
  } while (0)
  // prologue: K-tiles 0 and 1 in flight, K-tile 0 landed, first sets A0(0) B0(0) in registers
  stage_half(0, 0, 0);
  stage_half(0, 0, 1);
  stage_half(1, 1, 0);
  stage_half(1, 1, 1);
  wait_vm<16>();
  __builtin_amdgcn_s_barrier();
  ldA(0, 0);
  ldB(0, 0);
  for (int h = 0; h < nk; h += 2) {
    // ---- even K-tile h
    Q4_SEC(); ldB(h, 1); mm(0, 0); pace(0);
    Q4_SEC(); ldA(h, 1); mm(0, 1); pace(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if constexpr (!(SKIP & 2)) __builtin_amdgcn_s_barrier();
    Q4_SEC(); ldA(h + 1, 0); stage_half(h + 2, 0, 0); mm(1, 1); pace(1);
    Q4_SEC(); ldB(h + 1, 1); stage_half(h + 2, 0, 1); mm(1, 0); pace(1);
    // ---- odd K-tile h+1
    Q4_SEC(); ldB(h + 1, 0); mm(0, 1); pace(0);
    Q4_SEC(); ldA(h + 1, 1); mm(0, 0); pace(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if constexpr (!(SKIP & 2)) __builtin_amdgcn_s_barrier();
    Q4_SEC(); ldA(h + 2, 0); stage_half(h + 3, 1, 0); mm(1, 0); pace(1);
    Q4_SEC(); ldB(h + 2, 0); stage_half(h + 3, 1, 1); mm(1, 1); pace(1);
  }
#undef Q4_SEC
  wait_vm<0>();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    char* crow = (char*)p.c + (m0 + wr * 128 + (i >> 2) * 64 + (i & 3) * 16 + frow) * p.ldc * 2;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const f32x4 v0 = acc[i][j], v1 = acc[i][j + 1];
      bf16x8 o = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                  (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
      *(uint4*)(crow + (n0 + wc * 128 + (j >> 2) * 64 + ((j >> 1) & 1) * 32 + fq * 8) * 2) =
          __builtin_bit_cast(uint4, o);
    }
  }
}

// fp32 reference: C[m][n] = sum_k A[m][k] * B[n][k]
// ---------------------------------------------------------------------------------------------
// pt4v: pt4 (nt | sc1 write-through C stores, as the product's CMODE 2) with VALU-free load
// phases. Stamps (r3_20/r3_21) showed phase A's load segment ~550 cycles longer than phase B's
// with equal read counts: its head carried the buffer-parity VGPR address arithmetic (a 16-bit
// ds offset cannot reach the second 64 KB buffer) and the LDS-DMA 64-bit address math, and VALU
// at the head of a segment costs the un-prioritized wave ~90 cycles each (MI355X_MICROARCH.md,
// two waves per SIMD, item 6). V bits:
//   1: LDS = [A units of both buffers | B units of both buffers]: every fragment read is a fixed
//      per-lane VGPR + compile-time offset (< 64 KB); the K-tile body is instantiated per parity
//   2: LDS-DMA through buffer descriptors: per-tile SGPR base, K offset in soffset, fixed
//      per-lane voffset (no per-stage VALU)
//   4: C stores through SGPR soffsets (fixed per-lane voffset)
//   8: a tile's first MFMA of each accumulator takes a zero C operand (no v_mov zeroing)
template <int V>
__device__ constexpr int pt4v_uoff(int X, int buf, int q) {
  return (V & 1) ? X * 65536 + buf * 32768 + q * 16384 : buf * 65536 + X * 32768 + q * 16384;
}

template <bool STAMP, int V>
__global__ __launch_bounds__(512) void pt4v_kernel(const Args p) {
  constexpr int ROWB = 128, UNIT = 128 * ROWB;
  constexpr int NS = 4;
  __shared__ __attribute__((aligned(1024))) char smem[8 * UNIT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int nk = p.K / 64;
  const int my_tiles =
      ((int)blockIdx.x < ntiles) ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  if (my_tiles == 0) return;
  const int drow = lane >> 3, dpc = lane & 7;
  unsigned offA[2][2], offB[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ur = wave * 16 + i * 8 + drow;
    const int ch = (dpc ^ ((ur >> 1) & 7)) * 16;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int lr = (ur >> 6) * 128 + q * 64 + (ur & 63);
      offA[q][i] = (unsigned)(lr * p.lda * 2 + ch);
      const int lc = (ur >> 5) * 64 + q * 32 + t8_perm(ur & 31);
      offB[q][i] = (unsigned)(lc * p.ldb * 2 + ch);
    }
  }
  const char* baseA = nullptr;
  const char* baseB = nullptr;
  __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.a, 0, 0x7FFFFFF0, 0x00020000);
  __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.b, 0, 0x7FFFFFF0, 0x00020000);
  const __amdgpu_buffer_rsrc_t crc =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.c, 0, 0x7FFFFFF0, 0x00020000);
  int src_tile = -1;
  auto origin = [&](int ti, int64_t& m0, int64_t& n0) __attribute__((always_inline)) {
    const int wg = xcd_remap((int)blockIdx.x + ti * (int)gridDim.x, ntiles);
    lab_tile_mn(wg, p.M / 256, tiles_n, p.raster, m0, n0);
  };
  struct Cur { int ti, kt; };
  auto adv = [&](Cur& c) __attribute__((always_inline)) {
    if (c.ti == my_tiles - 1 && c.kt == nk - 1) return;
    if (++c.kt == nk) { c.kt = 0; ++c.ti; }
  };
  auto stage = [&](int which, int buf, Cur c) __attribute__((always_inline)) {
    if constexpr ((V & 512) != 0) {  // timing only: no LDS-DMA after the first two K-tiles
      if (c.ti > 0 || c.kt >= 2) return;
    }
    if (c.ti != src_tile) {
      int64_t m0, n0;
      origin(c.ti, m0, n0);
      baseA = (const char*)p.a + m0 * p.lda * 2;
      baseB = (const char*)p.b + n0 * p.ldb * 2;
      if constexpr ((V & 2) != 0) {
        rsA = __builtin_amdgcn_make_buffer_rsrc((void*)baseA, 0, 0x7FFFFFF0, 0x00020000);
        rsB = __builtin_amdgcn_make_buffer_rsrc((void*)baseB, 0, 0x7FFFFFF0, 0x00020000);
      }
      src_tile = c.ti;
    }
    const int X = which < 2 ? 0 : 1, q = which & 1;
    const unsigned* off = X == 0 ? offA[q] : offB[q];
    char* dst = smem + pt4v_uoff<V>(X, buf, q) + wave * 16 * ROWB;
    if constexpr ((V & 2) != 0) {
      const unsigned soff = (unsigned)(c.kt * ROWB);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(X == 0 ? rsA : rsB, (LDS_AS void*)dst, 16, off[0],
                                               soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(X == 0 ? rsA : rsB, (LDS_AS void*)(dst + 8 * ROWB),
                                               16, off[1], soff, 0, 0);
    } else {
      const char* base = (X == 0 ? baseA : baseB) + (int64_t)c.kt * ROWB;
      glds16(base + off[0], dst);
      glds16(base + off[1], dst + 8 * ROWB);
    }
  };
  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;
  const int c0 = ((0 + fq) ^ sw) * 16, c1 = ((4 + fq) ^ sw) * 16;
  const int aoff = (wr * 64 + frow) * ROWB, boff = (wc * 32 + frow) * ROWB;
  const unsigned rA0 = aoff + c0, rA1 = aoff + c1;
  const unsigned rB0 = ((V & 1) ? 0 : 0) + boff + c0, rB1 = boff + c1;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x4 aR[4][2], bR[2][2][2];
  auto loadA = [&](auto bufc, int mq) __attribute__((always_inline)) {
    constexpr int BUF = decltype(bufc)::value;
    if constexpr ((V & 128) != 0) return;  // timing only: no LDS reads
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int o = pt4v_uoff<V>(0, BUF, mq) + f * 16 * ROWB;
      aR[f][0] = *(const i32x4*)(smem + rA0 + o);
      aR[f][1] = *(const i32x4*)(smem + rA1 + o);
    }
  };
  auto loadB = [&](auto bufc, int nq) __attribute__((always_inline)) {
    constexpr int BUF = decltype(bufc)::value;
    if constexpr ((V & 128) != 0) return;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int o = pt4v_uoff<V>(1, BUF, nq) + g * 16 * ROWB;
      bR[nq][g][0] = *(const i32x4*)(smem + rB0 + o);
      bR[nq][g][1] = *(const i32x4*)(smem + rB1 + o);
    }
  };
  auto mm = [&](int mq, int nq, bool zero) __attribute__((always_inline)) {
    if constexpr ((V & 256) != 0) {  // timing only: no MFMA
#pragma unroll
      for (int f = 0; f < 4; ++f) asm volatile("" ::"v"(aR[f][0]), "v"(aR[f][1]), "v"(bR[nq][0][1]));
      return;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          f32x4& a = acc[mq * 4 + f][nq * 2 + g];
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, bR[nq][g][kk]), __builtin_bit_cast(bf16x8, aR[f][kk]),
              (zero && kk == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : a, 0, 0, 0);
        }
  };
  int ti = 0;
  const unsigned c_lane = (unsigned)(((wr * 128 + frow) * p.ldc + wc * 64 + fq * 8) * 2);
  auto store_frag = [&](int mq, int nq, int f, int sti) __attribute__((always_inline)) {
    const int i = mq * 4 + f;
    if constexpr ((V & 64) != 0) {  // timing only: no C stores
      asm volatile("" ::"v"(acc[i][nq * 2]), "v"(acc[i][nq * 2 + 1]));
      return;
    }
    int64_t m0, n0;
    origin(sti, m0, n0);
    const f32x4 v0 = acc[i][nq * 2], v1 = acc[i][nq * 2 + 1];
    bf16x8 o = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
    typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
    if constexpr ((V & 4) != 0) {
      const unsigned soff = (unsigned)(((m0 + mq * 64 + f * 16) * p.ldc + n0) * 2 + nq * 64);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), crc, c_lane, soff, 18);
    } else {
      char* crow = (char*)p.c + (m0 + wr * 128 + mq * 64 + f * 16 + frow) * p.ldc * 2;
      const char* dst = crow + (n0 + wc * 64 + nq * 32 + fq * 8) * 2;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), crc,
                                             (unsigned)(dst - (const char*)p.c), 0, 18);
    }
    if constexpr ((V & 8) == 0) {
      acc[i][nq * 2] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc[i][nq * 2 + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store_q = [&](int mq, int nq, int sti) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int f = 0; f < 4; ++f) store_frag(mq, nq, f, sti);
    __builtin_amdgcn_sched_barrier(0);
  };
#define T4_BAR()                         \
  do {                                   \
    __builtin_amdgcn_sched_barrier(0);   \
    __builtin_amdgcn_s_barrier();        \
    __builtin_amdgcn_sched_barrier(0);   \
  } while (0)
#define T4_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
  const bool g1 = wr == 1;
  unsigned long long st[16] = {}, tprev = 0;
  auto T = [&](int bucket) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
      if (bucket >= 0) st[bucket] += t - tprev;
      tprev = t;
    }
  };
  Cur q0{0, 0}, q1{0, 0};
  adv(q1);
  stage(2, 0, q0);
  stage(3, 0, q0);
  stage(0, 0, q0);
  stage(1, 0, q0);
  stage(2, 1, q1);
  stage(3, 1, q1);
  Cur qa = q1, qb = q1;
  adv(qb);
  wait_vm<6>();
  T4_BAR();
  if (g1) T4_BAR();
  T(-1);
  const unsigned long long t_start = tprev;
  // V & 1024: static priority (waves 4-7 at 1 for the whole kernel, no per-phase flips);
  // V & 4096: no s_setprio at all
  constexpr bool FLIP = (V & (1024 | 4096)) == 0;
  if constexpr ((V & 1024) != 0) {
    if (g1) __builtin_amdgcn_s_setprio(1);
  }
  auto iter = [&](auto bufc, auto kind_tag) __attribute__((always_inline)) {
    constexpr int KIND = decltype(kind_tag)::value;
    constexpr int BUF = decltype(bufc)::value;
    constexpr bool Z = (V & 8) != 0 && KIND == 2;
    if constexpr ((V & 2048) != 0) {  // the LDS-DMA pieces first, then the fragment reads
      stage(0, BUF ^ 1, qa);
      stage(1, BUF ^ 1, qa);
    }
    if constexpr ((V & 16) != 0) {  // timing only: phase A reads A0 + A1, phase B B0 + B1
      loadA(bufc, 0);
#pragma unroll
      for (int f = 0; f < 4; ++f) asm volatile("" ::"v"(aR[f][0]), "v"(aR[f][1]));
      loadA(bufc, 1);
    } else {
      loadB(bufc, 0);  // phase A
      loadB(bufc, 1);
      loadA(bufc, 0);
    }
    T(0);
    if constexpr ((V & 2048) == 0) {
      stage(0, BUF ^ 1, qa);
      stage(1, BUF ^ 1, qa);
    }
    T(1);
    T4_LGKM0();
    T(2);
    if (g1) wait_vm<KIND == 2 ? 8 + 4 * NS : 8>();
    T(6);
    T4_BAR();
    T(7);
    if constexpr (FLIP) __builtin_amdgcn_s_setprio(1);
    mm(0, 0, Z);
    mm(0, 1, Z);
    if constexpr (FLIP) __builtin_amdgcn_s_setprio(0);
    T(11);
    if constexpr (KIND == 1) { store_q(0, 0, ti); store_q(0, 1, ti); }
    T(13);
    if (!g1) wait_vm<KIND == 1 ? 8 + 2 * NS : (KIND == 2 ? 8 + 4 * NS : 8)>();
    T(6);
    T4_BAR();
    T(8);
    if constexpr ((V & 2048) != 0) {
      stage(2, BUF, qb);
      stage(3, BUF, qb);
    }
    if constexpr ((V & 16) != 0) {
      loadB(bufc, 0);
      loadB(bufc, 1);
    } else {
      loadA(bufc, 1);  // phase B
    }
    T(3);
    if constexpr ((V & 2048) == 0) {
      stage(2, BUF, qb);
      stage(3, BUF, qb);
    }
    T(4);
    T4_LGKM0();
    T(5);
    if (g1) wait_vm<KIND == 1 ? 6 + 2 * NS : 6>();
    T(6);
    T4_BAR();
    T(9);
    if constexpr (FLIP) __builtin_amdgcn_s_setprio(1);
    mm(1, 1, Z);
    mm(1, 0, Z);
    if constexpr (FLIP) __builtin_amdgcn_s_setprio(0);
    T(12);
    if constexpr (KIND == 1) { store_q(1, 1, ti); store_q(1, 0, ti); }
    T(13);
    if (!g1) wait_vm<KIND == 1 ? 6 + 4 * NS : 6>();
    T(6);
    T4_BAR();
    T(10);
    qa = qb;
    adv(qb);
  };
  // buffer parity is static by position: every tile has an even number (>= 4) of K-tiles, so
  // each tile starts in buffer 0 and its body is unrolled by two (a run-time parity branch
  // between two instantiations made the register allocator spill ~250 VGPRs)
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;
  auto tile_body = [&](auto first_kind) __attribute__((always_inline)) {
    iter(B0{}, first_kind);
    iter(B1{}, K0{});
    for (int t = 2; t < nk - 2; t += 2) {
      iter(B0{}, K0{});
      iter(B1{}, K0{});
    }
    iter(B0{}, K0{});
    iter(B1{}, K1{});
  };
  ti = 0;
  tile_body(K0{});
  for (ti = 1; ti < my_tiles; ++ti) tile_body(std::integral_constant<int, 2>{});
  if (!g1) T4_BAR();
#undef T4_BAR
#undef T4_LGKM0
  wait_vm<0>();
  if constexpr (STAMP) {
    T(-1);
    st[14] = tprev - t_start;
    if (lane == 0) {
      unsigned long long* o = p.stamps + ((size_t)blockIdx.x * 8 + wave) * 16;
#pragma unroll
      for (int j = 0; j < 15; ++j) o[j] = st[j];
      o[15] = (unsigned long long)my_tiles;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// pt4k: pt4v15 with the K-tile split by K HALVES instead of M / N halves: phase A reads the first
// 32 K of every fragment (8 A + 4 B ds_reads, 32 MFMAs), phase B the second 32 (the same), so the
// two load phases are equal (pt4: 16 / 8 reads). LDS regions (X, buf, h) of 256 rows x 64 B
// (X * 64K + buf * 32K + h * 16K; chunks swizzled by swz64); a region is restaged as soon as both
// wave groups have read it: phase A of K-tile t stages the h = 1 regions of t + 1, phase B the
// h = 0 regions of t + 2 (6 intervals of DMA lead for both). vmcnt: 8 per wait, + 16 (the tile's
// C stores, all issued after its last MFMA B) at the two waits behind them.
template <bool STAMP>
__global__ __launch_bounds__(512) void pt4k_kernel(const Args p) {
  constexpr int ROWB = 128, HB = 64;  // bytes per K-tile row / per K-half row
  constexpr int NSQ = 16;             // C store instructions per wave per tile (bf16)
  __shared__ __attribute__((aligned(1024))) char smem[131072];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int nk = p.K / 64;
  const int my_tiles =
      ((int)blockIdx.x < ntiles) ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  if (my_tiles == 0) return;
  // DMA: a wave fills rows wave * 32 .. + 31 of a region, 16 rows x 64 B per instruction
  const int drow = lane >> 2, dch = lane & 3;
  unsigned offA[2], offB[2];  // [i]; K half h adds h * 64 in the instruction's offset field
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = wave * 32 + i * 16 + drow;
    const int col = (r & ~31) + t8_perm(r & 31);
    const int ch = (dch ^ swz64(r)) * 16;
    offA[i] = (unsigned)(r * p.lda * 2 + ch);
    offB[i] = (unsigned)(col * p.ldb * 2 + ch);
  }
  __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.a, 0, 0x7FFFFFF0, 0x00020000);
  __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.b, 0, 0x7FFFFFF0, 0x00020000);
  const __amdgpu_buffer_rsrc_t crc =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.c, 0, 0x7FFFFFF0, 0x00020000);
  int src_tile = -1;
  auto origin = [&](int ti, int64_t& m0, int64_t& n0) __attribute__((always_inline)) {
    const int wg = xcd_remap((int)blockIdx.x + ti * (int)gridDim.x, ntiles);
    m0 = (int64_t)(wg / tiles_n) * 256;
    n0 = (int64_t)(wg % tiles_n) * 256;
  };
  struct Cur { int ti, kt; };
  auto adv = [&](Cur& c) __attribute__((always_inline)) {
    if (c.ti == my_tiles - 1 && c.kt == nk - 1) return;
    if (++c.kt == nk) { c.kt = 0; ++c.ti; }
  };
  auto reg = [](int X, int buf, int h) constexpr { return X * 65536 + buf * 32768 + h * 16384; };
  // both regions (A and B) of K-half h of K-tile c into buffer buf: 4 instructions per wave
  auto stage = [&](int buf, auto hc, Cur c) __attribute__((always_inline)) {
    constexpr int h = decltype(hc)::value;
    if (c.ti != src_tile) {
      int64_t m0, n0;
      origin(c.ti, m0, n0);
      rsA = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.a + m0 * p.lda * 2), 0,
                                              0x7FFFFFF0, 0x00020000);
      rsB = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.b + n0 * p.ldb * 2), 0,
                                              0x7FFFFFF0, 0x00020000);
      src_tile = c.ti;
    }
    const unsigned soff = (unsigned)(c.kt * ROWB);
#pragma unroll
    for (int X = 0; X < 2; ++X) {
      // the instruction offset (h * 64, the K half) moves the LDS destination too: start that
      // much lower so the 64-byte rows land in place
      char* dst = smem + reg(X, buf, h) + wave * 32 * HB - h * HB;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(X == 0 ? rsA : rsB,
                                                 (LDS_AS void*)(dst + i * 16 * HB), 16,
                                                 X == 0 ? offA[i] : offB[i], soff, h * HB, 0);
    }
  };
  const int frow = lane & 15, fq = lane >> 4;
  const int fch = (fq ^ swz64(frow)) * 16;
  unsigned rA = (wr * 128 + frow) * HB + fch, rB = 65536 + (wc * 64 + frow) * HB + fch;
  // opaque bases: otherwise the B base's 64K is re-associated into the per-read constant, which
  // then no longer fits the ds_read offset field (a VGPR per read, spilled)
  asm volatile("" : "+v"(rA), "+v"(rB));
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x4 aR[8], bR[4];
  auto load = [&](auto bufc, auto hc) __attribute__((always_inline)) {
    constexpr int BUF = decltype(bufc)::value, H = decltype(hc)::value;
#pragma unroll
    for (int g = 0; g < 4; ++g) bR[g] = *(const i32x4*)(smem + rB + reg(0, BUF, H) + g * 16 * HB);
#pragma unroll
    for (int f = 0; f < 8; ++f) aR[f] = *(const i32x4*)(smem + rA + reg(0, BUF, H) + f * 16 * HB);
  };
  auto mm = [&](bool zero) __attribute__((always_inline)) {
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(bf16x8, bR[g]), __builtin_bit_cast(bf16x8, aR[f]),
            zero ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[f][g], 0, 0, 0);
  };
  int ti = 0;
  const unsigned c_lane = (unsigned)(((wr * 128 + frow) * p.ldc + wc * 64 + fq * 8) * 2);
  auto store_tile = [&]() __attribute__((always_inline)) {
    int64_t m0, n0;
    origin(ti, m0, n0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
      for (int nq = 0; nq < 2; ++nq) {
        const f32x4 v0 = acc[f][nq * 2], v1 = acc[f][nq * 2 + 1];
        bf16x8 o = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                    (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
        typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
        const unsigned soff = (unsigned)(((m0 + f * 16) * p.ldc + n0) * 2 + nq * 64);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), crc, c_lane, soff, 18);
      }
    __builtin_amdgcn_sched_barrier(0);
  };
#define T4_BAR()                         \
  do {                                   \
    __builtin_amdgcn_sched_barrier(0);   \
    __builtin_amdgcn_s_barrier();        \
    __builtin_amdgcn_sched_barrier(0);   \
  } while (0)
#define T4_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
  const bool g1 = wr == 1;
  unsigned long long st[16] = {}, tprev = 0;
  auto T = [&](int bucket) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
      if (bucket >= 0) st[bucket] += t - tprev;
      tprev = t;
    }
  };
  using H0 = std::integral_constant<int, 0>;
  using H1 = std::integral_constant<int, 1>;
  Cur q0{0, 0}, q1{0, 0};
  adv(q1);
  stage(0, H0{}, q0);  // "D_B(-2)": K-tile 0, h = 0
  stage(0, H1{}, q0);  // "D_A(-1)": K-tile 0, h = 1
  stage(1, H0{}, q1);  // "D_B(-1)": K-tile 1, h = 0
  Cur qa = q1, qb = q1;  // qa: K-tile t + 1 (phase A stages its h = 1), qb: t + 2 (h = 0)
  adv(qb);
  wait_vm<8>();
  T4_BAR();
  if (g1) T4_BAR();
  T(-1);
  const unsigned long long t_start = tprev;
  auto iter = [&](auto bufc, auto kind_tag) __attribute__((always_inline)) {
    constexpr int KIND = decltype(kind_tag)::value;
    constexpr int BUF = decltype(bufc)::value;
    constexpr bool Z = KIND == 2;
    load(bufc, H0{});  // phase A: K half 0
    T(0);
    stage(BUF ^ 1, H1{}, qa);
    T(1);
    T4_LGKM0();
    T(2);
    if (g1) wait_vm<KIND == 2 ? 8 + NSQ : 8>();
    T(6);
    T4_BAR();
    T(7);
    __builtin_amdgcn_s_setprio(1);
    mm(Z);
    __builtin_amdgcn_s_setprio(0);
    T(11);
    if (!g1) wait_vm<KIND == 2 ? 8 + NSQ : 8>();
    T(6);
    T4_BAR();
    T(8);
    load(bufc, H1{});  // phase B: K half 1
    T(3);
    stage(BUF, H0{}, qb);
    T(4);
    T4_LGKM0();
    T(5);
    if (g1) wait_vm<8>();
    T(6);
    T4_BAR();
    T(9);
    __builtin_amdgcn_s_setprio(1);
    mm(false);
    __builtin_amdgcn_s_setprio(0);
    T(12);
    if constexpr (KIND == 1) store_tile();
    T(13);
    if (!g1) wait_vm<KIND == 1 ? 8 + NSQ : 8>();
    T(6);
    T4_BAR();
    T(10);
    qa = qb;
    adv(qb);
  };
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;
  auto tile_body = [&](auto first_kind) __attribute__((always_inline)) {
    iter(B0{}, first_kind);
    for (int t = 1; t + 2 < nk; t += 2) {
      iter(B1{}, K0{});
      iter(B0{}, K0{});
    }
    iter(B1{}, K1{});
  };
  ti = 0;
  tile_body(K0{});
  for (ti = 1; ti < my_tiles; ++ti) tile_body(std::integral_constant<int, 2>{});
  if (!g1) T4_BAR();
#undef T4_BAR
#undef T4_LGKM0
  wait_vm<0>();
  if constexpr (STAMP) {
    T(-1);
    st[14] = tprev - t_start;
    if (lane == 0) {
      unsigned long long* o = p.stamps + ((size_t)blockIdx.x * 8 + wave) * 16;
#pragma unroll
      for (int j = 0; j < 15; ++j) o[j] = st[j];
      o[15] = (unsigned long long)my_tiles;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// pt4d: pt4v15 with balanced load phases on 128-byte-row units. Phase A of K-tile t reads the
// first halves (A rows mq = 0, B cols nq = 0: 8 + 4 ds_reads) and computes A0 x B0 plus the
// DEFERRED A1 x B1 of K-tile t - 1 (its fragments are still in registers); phase B reads the
// second halves (8 + 4) and computes A0 x B1 + A1 x B0. A tile's last K-tile does its own A1 x B1
// in phase B. Fragments of both halves stay live (96 VGPRs). A unit is restaged as soon as both
// wave groups have read it (phase A(t): halves 1 of K-tile t + 1; phase B(t): halves 0 of t + 2),
// so every unit gets 6 intervals of DMA lead. KIND 0 normal, 1 last, 2 first after a tile,
// 4 first of the kernel (no deferred product, no store counts).
template <bool STAMP, bool PRIO = true, int STS = 0>
__global__ __launch_bounds__(512) void pt4d_kernel(const Args p) {
  constexpr int ROWB = 128, UNIT = 128 * ROWB;
  constexpr int NS = 4;  // C store instructions per quadrant per wave (bf16)
  __shared__ __attribute__((aligned(1024))) char smem[8 * UNIT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int nk = p.K / 64;
  const int my_tiles =
      ((int)blockIdx.x < ntiles) ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  if (my_tiles == 0) return;
  const int drow = lane >> 3, dpc = lane & 7;
  unsigned offA[2][2], offB[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ur = wave * 16 + i * 8 + drow;
    const int ch = (dpc ^ ((ur >> 1) & 7)) * 16;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int lr = (ur >> 6) * 128 + q * 64 + (ur & 63);
      offA[q][i] = (unsigned)(lr * p.lda * 2 + ch);
      const int lc = (ur >> 5) * 64 + q * 32 + t8_perm(ur & 31);
      offB[q][i] = (unsigned)(lc * p.ldb * 2 + ch);
    }
  }
  const __amdgpu_buffer_rsrc_t crc =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.c, 0, 0x7FFFFFF0, 0x00020000);
  __amdgpu_buffer_rsrc_t rsA = crc, rsB = crc;
  int src_tile = -1;
  auto origin = [&](int ti, int64_t& m0, int64_t& n0) __attribute__((always_inline)) {
    const int wg = xcd_remap((int)blockIdx.x + ti * (int)gridDim.x, ntiles);
    lab_tile_mn(wg, p.M / 256, tiles_n, p.raster, m0, n0);
  };
  int64_t cm0 = 0, cn0 = 0, nm0 = 0, nn0 = 0;
  origin(0, nm0, nn0);
  struct Cur { int ti, kt; };
  auto adv = [&](Cur& c) __attribute__((always_inline)) {
    if (c.ti == my_tiles - 1 && c.kt == nk - 1) return;
    if (++c.kt == nk) { c.kt = 0; ++c.ti; }
  };
  auto uoff = [](int X, int buf, int q) constexpr { return X * 65536 + buf * 32768 + q * 16384; };
  auto stage = [&](int X, int q, int buf, Cur c) __attribute__((always_inline)) {
    if (c.ti != src_tile) {
      rsA = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.a + nm0 * p.lda * 2), 0,
                                              0x7FFFFFF0, 0x00020000);
      rsB = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.b + nn0 * p.ldb * 2), 0,
                                              0x7FFFFFF0, 0x00020000);
      src_tile = c.ti;
    }
    const unsigned* off = X == 0 ? offA[q] : offB[q];
    char* dst = smem + uoff(X, buf, q) + wave * 16 * ROWB;
    const unsigned soff = (unsigned)(c.kt * ROWB);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(X == 0 ? rsA : rsB, (LDS_AS void*)dst, 16, off[0],
                                             soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(X == 0 ? rsA : rsB, (LDS_AS void*)(dst + 8 * ROWB),
                                             16, off[1], soff, 0, 0);
  };
  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;
  const int c0 = ((0 + fq) ^ sw) * 16, c1 = ((4 + fq) ^ sw) * 16;
  unsigned rA0 = (wr * 64 + frow) * ROWB + c0, rA1 = (wr * 64 + frow) * ROWB + c1;
  unsigned rB0 = 65536 + (wc * 32 + frow) * ROWB + c0, rB1 = 65536 + (wc * 32 + frow) * ROWB + c1;
  asm volatile("" : "+v"(rA0), "+v"(rA1), "+v"(rB0), "+v"(rB1));
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x4 aX[2][4][2], bX[2][2][2];  // [half][frag][k16]
  auto loadA = [&](auto bufc, int mq) __attribute__((always_inline)) {
    constexpr int BUF = decltype(bufc)::value;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int o = uoff(0, BUF, mq) + f * 16 * ROWB;
      aX[mq][f][0] = *(const i32x4*)(smem + rA0 + o);
      aX[mq][f][1] = *(const i32x4*)(smem + rA1 + o);
    }
  };
  auto loadB = [&](auto bufc, int nq) __attribute__((always_inline)) {
    constexpr int BUF = decltype(bufc)::value;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int o = uoff(0, BUF, nq) + g * 16 * ROWB;
      bX[nq][g][0] = *(const i32x4*)(smem + rB0 + o);
      bX[nq][g][1] = *(const i32x4*)(smem + rB1 + o);
    }
  };
  auto mm = [&](int mq, int nq, bool zero) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          f32x4& a = acc[mq * 4 + f][nq * 2 + g];
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, bX[nq][g][kk]), __builtin_bit_cast(bf16x8, aX[mq][f][kk]),
              (zero && kk == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : a, 0, 0, 0);
        }
  };
  int ti = 0;
  const unsigned c_lane = (unsigned)(((wr * 128 + frow) * p.ldc + wc * 64 + fq * 8) * 2);
  auto store_q = [&](int mq, int nq) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int i = mq * 4 + f;
      const f32x4 v0 = acc[i][nq * 2], v1 = acc[i][nq * 2 + 1];
      bf16x8 o = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                  (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
      typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
      if constexpr (STS == 2) {  // timing only: 32 rows x 32 B per instruction (wrong layout)
        const int row = wr * 128 + mq * 64 + (f >> 1) * 32 + (lane & 31);
        const int col = wc * 64 + nq * 32 + (f & 1) * 16 + (lane >> 5) * 8;
        const unsigned voff = (unsigned)((row * p.ldc + col) * 2);
        const unsigned soff = (unsigned)((cm0 * p.ldc + cn0) * 2);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), crc, voff, soff, 18);
      } else {
        const unsigned soff = (unsigned)(((cm0 + mq * 64 + f * 16) * p.ldc + cn0) * 2 + nq * 64);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), crc, c_lane, soff, 18);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
#define T4_BAR()                         \
  do {                                   \
    __builtin_amdgcn_sched_barrier(0);   \
    __builtin_amdgcn_s_barrier();        \
    __builtin_amdgcn_sched_barrier(0);   \
  } while (0)
#define T4_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
  const bool g1 = wr == 1;
  Cur q0{0, 0}, q1{0, 0};
  adv(q1);
  stage(0, 0, 0, q0);  // halves 0 of K-tile 0
  stage(1, 0, 0, q0);
  stage(0, 1, 0, q0);  // halves 1 of K-tile 0
  stage(1, 1, 0, q0);
  stage(0, 0, 1, q1);  // halves 0 of K-tile 1
  stage(1, 0, 1, q1);
  Cur qa = q1, qb = q1;  // qa: K-tile t + 1 (halves 1, phase A), qb: t + 2 (halves 0, phase B)
  adv(qb);
  wait_vm<8>();
  T4_BAR();
  if (g1) T4_BAR();
  auto iter = [&](auto bufc, auto kind_tag) __attribute__((always_inline)) {
    constexpr int KIND = decltype(kind_tag)::value;
    constexpr int BUF = decltype(bufc)::value;
    constexpr bool Z = KIND == 2 || KIND == 4;
    constexpr bool DEF = KIND == 0 || KIND == 1;  // the previous K-tile's A1 x B1
    loadB(bufc, 0);  // phase A: halves 0
    loadA(bufc, 0);
    stage(0, 1, BUF ^ 1, qa);
    stage(1, 1, BUF ^ 1, qa);
    T4_LGKM0();
    if (g1) wait_vm<KIND == 2 ? 8 + 3 * NS : 8>();
    T4_BAR();
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
    if constexpr (DEF) mm(1, 1, false);
    mm(0, 0, Z);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    if constexpr (KIND == 1) store_q(0, 0);
    if (!g1) wait_vm<KIND == 2 ? 8 + 3 * NS : (KIND == 1 ? 8 + NS : 8)>();
    T4_BAR();
    loadB(bufc, 1);  // phase B: halves 1
    loadA(bufc, 1);
    stage(0, 0, BUF, qb);
    stage(1, 0, BUF, qb);
    T4_LGKM0();
    if (g1) wait_vm<KIND == 1 ? 8 + NS : 8>();
    T4_BAR();
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
    mm(0, 1, Z);
    mm(1, 0, Z);
    if constexpr (KIND == 1) mm(1, 1, false);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    if constexpr (KIND == 1) {
      store_q(0, 1);
      store_q(1, 0);
      store_q(1, 1);
#pragma unroll
      for (int f = 0; f < 4; ++f) {  // quadrant (1, 1)'s first MFMA of the next tile is deferred
        acc[4 + f][2] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc[4 + f][3] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    if (!g1) wait_vm<KIND == 1 ? 8 + 4 * NS : 8>();
    T4_BAR();
    qa = qb;
    adv(qb);
  };
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;
  auto tile_body = [&](auto first_kind) __attribute__((always_inline)) {
    cm0 = nm0;
    cn0 = nn0;
    if (ti + 1 < my_tiles) origin(ti + 1, nm0, nn0);
    iter(B0{}, first_kind);
    for (int t = 1; t + 2 < nk; t += 2) {
      iter(B1{}, K0{});
      iter(B0{}, K0{});
    }
    iter(B1{}, K1{});
  };
  ti = 0;
  tile_body(std::integral_constant<int, 4>{});
  for (ti = 1; ti < my_tiles; ++ti) tile_body(std::integral_constant<int, 2>{});
  if (!g1) T4_BAR();
#undef T4_BAR
#undef T4_LGKM0
  wait_vm<0>();
}

// ---------------------------------------------------------------------------------------------
// pt4e: pt4d whose second-half fragment reads move into the MFMA phase A (behind the deferred
// A1 x B1, interleaved with A0 x B0), so load phase B carries only LDS-DMA. Waits move one
// interval earlier for the halves 1 (5 intervals of DMA lead). Derived from:
// pt4d: pt4v15 with balanced load phases on 128-byte-row units. Phase A of K-tile t reads the
// first halves (A rows mq = 0, B cols nq = 0: 8 + 4 ds_reads) and computes A0 x B0 plus the
// DEFERRED A1 x B1 of K-tile t - 1 (its fragments are still in registers); phase B reads the
// second halves (8 + 4) and computes A0 x B1 + A1 x B0. A tile's last K-tile does its own A1 x B1
// in phase B. Fragments of both halves stay live (96 VGPRs). A unit is restaged as soon as both
// wave groups have read it (phase A(t): halves 1 of K-tile t + 1; phase B(t): halves 0 of t + 2),
// so every unit gets 6 intervals of DMA lead. KIND 0 normal, 1 last, 2 first after a tile,
// 4 first of the kernel (no deferred product, no store counts).
template <bool STAMP>
__global__ __launch_bounds__(512) void pt4e_kernel(const Args p) {
  constexpr int ROWB = 128, UNIT = 128 * ROWB;
  constexpr int NS = 4;  // C store instructions per quadrant per wave (bf16)
  __shared__ __attribute__((aligned(1024))) char smem[8 * UNIT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int nk = p.K / 64;
  const int my_tiles =
      ((int)blockIdx.x < ntiles) ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  if (my_tiles == 0) return;
  const int drow = lane >> 3, dpc = lane & 7;
  unsigned offA[2][2], offB[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ur = wave * 16 + i * 8 + drow;
    const int ch = (dpc ^ ((ur >> 1) & 7)) * 16;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int lr = (ur >> 6) * 128 + q * 64 + (ur & 63);
      offA[q][i] = (unsigned)(lr * p.lda * 2 + ch);
      const int lc = (ur >> 5) * 64 + q * 32 + t8_perm(ur & 31);
      offB[q][i] = (unsigned)(lc * p.ldb * 2 + ch);
    }
  }
  const __amdgpu_buffer_rsrc_t crc =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.c, 0, 0x7FFFFFF0, 0x00020000);
  __amdgpu_buffer_rsrc_t rsA = crc, rsB = crc;
  int src_tile = -1;
  auto origin = [&](int ti, int64_t& m0, int64_t& n0) __attribute__((always_inline)) {
    const int wg = xcd_remap((int)blockIdx.x + ti * (int)gridDim.x, ntiles);
    lab_tile_mn(wg, p.M / 256, tiles_n, p.raster, m0, n0);
  };
  int64_t cm0 = 0, cn0 = 0, nm0 = 0, nn0 = 0;
  origin(0, nm0, nn0);
  struct Cur { int ti, kt; };
  auto adv = [&](Cur& c) __attribute__((always_inline)) {
    if (c.ti == my_tiles - 1 && c.kt == nk - 1) return;
    if (++c.kt == nk) { c.kt = 0; ++c.ti; }
  };
  auto uoff = [](int X, int buf, int q) constexpr { return X * 65536 + buf * 32768 + q * 16384; };
  auto stage = [&](int X, int q, int buf, Cur c) __attribute__((always_inline)) {
    if (c.ti != src_tile) {
      rsA = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.a + nm0 * p.lda * 2), 0,
                                              0x7FFFFFF0, 0x00020000);
      rsB = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.b + nn0 * p.ldb * 2), 0,
                                              0x7FFFFFF0, 0x00020000);
      src_tile = c.ti;
    }
    const unsigned* off = X == 0 ? offA[q] : offB[q];
    char* dst = smem + uoff(X, buf, q) + wave * 16 * ROWB;
    const unsigned soff = (unsigned)(c.kt * ROWB);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(X == 0 ? rsA : rsB, (LDS_AS void*)dst, 16, off[0],
                                             soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(X == 0 ? rsA : rsB, (LDS_AS void*)(dst + 8 * ROWB),
                                             16, off[1], soff, 0, 0);
  };
  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;
  const int c0 = ((0 + fq) ^ sw) * 16, c1 = ((4 + fq) ^ sw) * 16;
  unsigned rA0 = (wr * 64 + frow) * ROWB + c0, rA1 = (wr * 64 + frow) * ROWB + c1;
  unsigned rB0 = 65536 + (wc * 32 + frow) * ROWB + c0, rB1 = 65536 + (wc * 32 + frow) * ROWB + c1;
  asm volatile("" : "+v"(rA0), "+v"(rA1), "+v"(rB0), "+v"(rB1));
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x4 aX[2][4][2], bX[2][2][2];  // [half][frag][k16]
  auto loadA = [&](auto bufc, int mq) __attribute__((always_inline)) {
    constexpr int BUF = decltype(bufc)::value;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int o = uoff(0, BUF, mq) + f * 16 * ROWB;
      aX[mq][f][0] = *(const i32x4*)(smem + rA0 + o);
      aX[mq][f][1] = *(const i32x4*)(smem + rA1 + o);
    }
  };
  auto loadB = [&](auto bufc, int nq) __attribute__((always_inline)) {
    constexpr int BUF = decltype(bufc)::value;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int o = uoff(0, BUF, nq) + g * 16 * ROWB;
      bX[nq][g][0] = *(const i32x4*)(smem + rB0 + o);
      bX[nq][g][1] = *(const i32x4*)(smem + rB1 + o);
    }
  };
  auto mm = [&](int mq, int nq, bool zero) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          f32x4& a = acc[mq * 4 + f][nq * 2 + g];
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, bX[nq][g][kk]), __builtin_bit_cast(bf16x8, aX[mq][f][kk]),
              (zero && kk == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : a, 0, 0, 0);
        }
  };
  int ti = 0;
  const unsigned c_lane = (unsigned)(((wr * 128 + frow) * p.ldc + wc * 64 + fq * 8) * 2);
  auto store_q = [&](int mq, int nq) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int i = mq * 4 + f;
      const f32x4 v0 = acc[i][nq * 2], v1 = acc[i][nq * 2 + 1];
      bf16x8 o = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                  (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
      typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
      const unsigned soff = (unsigned)(((cm0 + mq * 64 + f * 16) * p.ldc + cn0) * 2 + nq * 64);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), crc, c_lane, soff, 18);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
#define T4_BAR()                         \
  do {                                   \
    __builtin_amdgcn_sched_barrier(0);   \
    __builtin_amdgcn_s_barrier();        \
    __builtin_amdgcn_sched_barrier(0);   \
  } while (0)
// lgkmcnt(0) as the builtin (vmcnt / expcnt at their maxima): the compiler's waitcnt pass sees
// it, so it does not re-wait for the load phase's reads inside the interleaved MFMA phase
#define T4_LGKM0() __builtin_amdgcn_s_waitcnt(0xC07F)
  const bool g1 = wr == 1;
  Cur q0{0, 0}, q1{0, 0};
  adv(q1);
  stage(0, 0, 0, q0);  // halves 0 of K-tile 0
  stage(1, 0, 0, q0);
  stage(0, 1, 0, q0);  // halves 1 of K-tile 0
  stage(1, 1, 0, q0);
  stage(0, 0, 1, q1);  // halves 0 of K-tile 1
  stage(1, 0, 1, q1);
  Cur qa = q1, qb = q1;  // qa: K-tile t + 1 (halves 1, phase A), qb: t + 2 (halves 0, phase B)
  adv(qb);
  wait_vm<8>();
  T4_BAR();
  if (g1) {  // g1's halves 1 of K-tile 0 are read in its first MFMA phase
    wait_vm<4>();
    T4_BAR();
  }
  auto iter = [&](auto bufc, auto kind_tag) __attribute__((always_inline)) {
    constexpr int KIND = decltype(kind_tag)::value;
    constexpr int BUF = decltype(bufc)::value;
    constexpr bool Z = KIND == 2 || KIND == 4;
    constexpr bool DEF = KIND == 0 || KIND == 1;  // the previous K-tile's A1 x B1
    loadB(bufc, 0);  // load phase A: halves 0
    loadA(bufc, 0);
    stage(0, 1, BUF ^ 1, qa);
    stage(1, 1, BUF ^ 1, qa);
    T4_LGKM0();
    // the halves 1 of this K-tile are read in the next interval (MFMA A) by this group
    if (!g1) wait_vm<KIND == 2 ? 8 + 4 * NS : 8>();
    T4_BAR();
    __builtin_amdgcn_s_setprio(1);
    if constexpr (DEF) mm(1, 1, false);  // frees the halves-1 registers
    __builtin_amdgcn_sched_barrier(0);
    loadB(bufc, 1);  // halves 1, interleaved with A0 x B0
    loadA(bufc, 1);
    mm(0, 0, Z);
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one ds_read
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    if constexpr (KIND == 1) store_q(0, 0);
    T4_LGKM0();
    T4_BAR();
    stage(0, 0, BUF, qb);  // load phase B: LDS-DMA only
    stage(1, 0, BUF, qb);
    if (g1) wait_vm<KIND == 1 ? 8 + NS : 8>();
    T4_BAR();
    __builtin_amdgcn_s_setprio(1);
    mm(0, 1, Z);
    mm(1, 0, Z);
    if constexpr (KIND == 1) mm(1, 1, false);
    __builtin_amdgcn_s_setprio(0);
    if constexpr (KIND == 1) {
      store_q(0, 1);
      store_q(1, 0);
      store_q(1, 1);
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        acc[4 + f][2] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc[4 + f][3] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    // g0: the halves 0 of the next K-tile (its next load phase); g1: the halves 1 of the next
    // K-tile, which g0 reads in the interval after this one
    if (!g1) wait_vm<KIND == 1 ? 8 + 4 * NS : 8>();
    else wait_vm<KIND == 1 ? 4 + 4 * NS : 4>();
    T4_BAR();
    qa = qb;
    adv(qb);
  };
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;
  auto tile_body = [&](auto first_kind) __attribute__((always_inline)) {
    cm0 = nm0;
    cn0 = nn0;
    if (ti + 1 < my_tiles) origin(ti + 1, nm0, nn0);
    iter(B0{}, first_kind);
    for (int t = 1; t + 2 < nk; t += 2) {
      iter(B1{}, K0{});
      iter(B0{}, K0{});
    }
    iter(B1{}, K1{});
  };
  ti = 0;
  tile_body(std::integral_constant<int, 4>{});
  for (ti = 1; ti < my_tiles; ++ti) tile_body(std::integral_constant<int, 2>{});
  if (!g1) T4_BAR();
#undef T4_BAR
#undef T4_LGKM0
  wait_vm<0>();
}

__global__ void ref_kernel(const __hip_bfloat16* A, const __hip_bfloat16* B, float* C, int M, int N,
                           int K) {
  __shared__ float as[16][65], bs[16][65];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m = blockIdx.y * 16 + ty, n = blockIdx.x * 16 + tx;
  float acc = 0.f;
  for (int k0 = 0; k0 < K; k0 += 64) {
    for (int kk = tx; kk < 64; kk += 16) {
      as[ty][kk] = (float)A[(size_t)(blockIdx.y * 16 + ty) * K + k0 + kk];
      bs[ty][kk] = (float)B[(size_t)(blockIdx.x * 16 + ty) * K + k0 + kk];
    }
    __syncthreads();
    for (int kk = 0; kk < 64; ++kk) acc += as[ty][kk] * bs[tx][kk];
    __syncthreads();
  }
  C[(size_t)m * N + n] = acc;
}

__global__ void fill_kernel(__hip_bfloat16* x, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    x[i] = (__hip_bfloat16)(((h & 0xffffff) / 16777216.0f) * 2.f - 1.f);
  }
}

__global__ void cmp_kernel(const __hip_bfloat16* C, const float* R, size_t n, float* maxerr) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  float e = 0.f;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) e = fmaxf(e, fabsf((float)C[i] - R[i]));
  atomicMax((int*)maxerr, __float_as_int(e));
}

typedef void (*KFn)(const Args);

struct Variant {
  const char* name;
  KFn fn;
  int ns;
  int threads;
  int all_tiles = 0;  // 1: one workgroup per tile (non-persistent)
};

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 65536;
  const int N = argc > 2 ? atoi(argv[2]) : 1024;
  const int K = argc > 3 ? atoi(argv[3]) : 1024;
  const int rounds = 5, iters = 20;
  if (M % 256 || N % 256 || K % 64) { fprintf(stderr, "shape must be multiple of 256/256/64\n"); return 2; }
  int dev = 0, ncu = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  __hip_bfloat16 *A, *B, *C;
  float *R, *err;
  CHECK(hipMalloc(&A, (size_t)M * K * 2));
  CHECK(hipMalloc(&B, (size_t)N * K * 2));
  CHECK(hipMalloc(&C, (size_t)M * N * 2));
  CHECK(hipMalloc(&R, (size_t)M * N * 4));
  CHECK(hipMalloc(&err, 4));
  fill_kernel<<<1024, 256>>>(A, (size_t)M * K, 1u);
  fill_kernel<<<1024, 256>>>(B, (size_t)N * K, 2u);
  ref_kernel<<<dim3(N / 16, M / 16), 256>>>(A, B, R, M, N, K);
  CHECK(hipDeviceSynchronize());
  unsigned long long* stamps;
  const int grid = std::min(ncu, (M / 256) * (N / 256));
  CHECK(hipMalloc(&stamps, ((size_t)grid * 8 * 16 + 8) * 8));

  Variant vs[] = {
      {"ring2 dmaAC", ring2_kernel<4, false, 2>, 4, 512, 0},
      {"t8", t8_kernel<false>, 2, 512, 1},
      {"pt8", pt8_kernel<false>, 2, 512, 0},
      {"t8b", t8b_kernel<false>, 2, 512, 1},
      {"t4", t4_kernel<false>, 2, 512, 1},
      {"pt4", pt4_kernel<false>, 2, 512, 0},
      {"pt4b", pt4b_kernel<false>, 2, 512, 0},
      {"pt4 noDMA", pt4_kernel<false, 1>, 2, 512, 0},
      {"pt4 noMFMA", pt4_kernel<false, 4>, 2, 512, 0},
      {"pt4 nt", pt4_kernel<false, 16>, 2, 512, 0},
      {"pt4 nt bal", pt4_kernel<false, 16 | 65536>, 2, 512, 0},
      {"pt4v0", pt4v_kernel<false, 0>, 2, 512, 0},
      {"pt4v1", pt4v_kernel<false, 1>, 2, 512, 0},
      {"pt4v3", pt4v_kernel<false, 3>, 2, 512, 0},
      {"pt4v7", pt4v_kernel<false, 7>, 2, 512, 0},
      {"pt4v15", pt4v_kernel<false, 15>, 2, 512, 0},
      {"pt4v15 AfirstBsecond", pt4v_kernel<false, 31>, 2, 512, 0},
      {"pt4k", pt4k_kernel<false>, 2, 512, 0},
      {"pt4d", pt4d_kernel<false>, 2, 512, 0},
      {"pt4e", pt4e_kernel<false>, 2, 512, 0},
      {"pt4d noprio", pt4d_kernel<false, false>, 2, 512, 0},
      {"pt4d st32x32", pt4d_kernel<false, true, 2>, 2, 512, 0},
      {"pt4v15 staticprio", pt4v_kernel<false, 15 | 1024>, 2, 512, 0},
      {"pt4v15 noprio", pt4v_kernel<false, 15 | 4096>, 2, 512, 0},
      {"pt4v15 dmafirst", pt4v_kernel<false, 15 | 2048>, 2, 512, 0},
      {"pt4v15 noST", pt4v_kernel<false, 15 | 64>, 2, 512, 0},
      {"pt4v15 noLDSrd", pt4v_kernel<false, 15 | 128>, 2, 512, 0},
      {"pt4v15 noMFMA", pt4v_kernel<false, 15 | 256>, 2, 512, 0},
      {"pt4v15 noDMA", pt4v_kernel<false, 15 | 512>, 2, 512, 0},
      {"pt4v15 noDMA noST", pt4v_kernel<false, 15 | 512 | 64>, 2, 512, 0},
      {"pt4v15 MFMA only", pt4v_kernel<false, 15 | 512 | 64 | 128>, 2, 512, 0},
      {"pt4 nt stag2", pt4_kernel<false, 16 | 64>, 2, 512, 0},
      {"pt4 nt stag6", pt4_kernel<false, 16 | 128>, 2, 512, 0},
      {"pt4 nt stag4ph", pt4_kernel<false, 16 | 192>, 2, 512, 0},
      {"pt4 nt noST", pt4_kernel<false, 16 | 2>, 2, 512, 0},
      {"pt4 nt ils", pt4_kernel<false, 16 | 256>, 2, 512, 0},
      {"pt4 nt noprio", pt4_kernel<false, 16 | 2048>, 2, 512, 0},
      {"pt4 nt bufdma", pt4_kernel<false, 16 | 8192>, 2, 512, 0},
      {"pt4 nt loadprio", pt4_kernel<false, 16 | 4096>, 2, 512, 0},
      {"pt4 nt ils free", pt4_kernel<false, 16 | 256 | 1024>, 2, 512, 0},
      {"pt4 nt smallC", pt4_kernel<false, 16 | 512>, 2, 512, 0},
      {"pt4 smallC", pt4_kernel<false, 512>, 2, 512, 0},
      {"pt4 fullline", pt4_kernel<false, 32>, 2, 512, 0},
      {"pt4 fullline nt", pt4_kernel<false, 48>, 2, 512, 0},
      {"pt4 noST", pt4_kernel<false, 2>, 2, 512, 0},
      {"pt4 noLDSrd", pt4_kernel<false, 8>, 2, 512, 0},
      {"pt4 noDMA noST", pt4_kernel<false, 3>, 2, 512, 0},
      {"pt4 noDMA noST noLDSrd", pt4_kernel<false, 11>, 2, 512, 0},
      {"pt4 wt", pt4_kernel<false, 16384>, 2, 512, 0},
      {"pt4 wt nt", pt4_kernel<false, 16384 | 16>, 2, 512, 0},
      {"pt4 sc01", pt4_kernel<false, 32768>, 2, 512, 0},
      {"q4", q4_kernel<0>, 2, 256, 1},
      {"q4 bufdma", q4_kernel<0, 8>, 2, 256, 1},
      {"q4s1 bufdma", q4_kernel<1, 8>, 2, 256, 1},
      {"q4 noDMA", q4_kernel<0, 1>, 2, 256, 1},
      {"q4 noBAR", q4_kernel<0, 2>, 2, 256, 1},
      {"q4 noDMA noBAR", q4_kernel<0, 3>, 2, 256, 1},
      {"q4 noMFMA", q4_kernel<0, 4>, 2, 256, 1},
  };
  Args a{A, B, C, K, K, N, M, N, K, nullptr, getenv("LAB_RASTER") ? atoi(getenv("LAB_RASTER")) : 0};
  const char* only = getenv("LAB_ONLY");  // comma-separated variant names: skip the others
  auto skip = [&](const char* name) {
    if (!only) return false;
    const size_t n = strlen(name);
    for (const char* q = only; *q;) {
      const char* e = strchr(q, ',');
      const size_t l = e ? (size_t)(e - q) : strlen(q);
      if (l == n && strncmp(q, name, n) == 0) return false;
      if (!e) break;
      q = e + 1;
    }
    return true;
  };
  const double flop = 2.0 * M * N * K;
  std::vector<std::vector<float>> times(sizeof(vs) / sizeof(vs[0]));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (size_t v = 0; v < sizeof(vs) / sizeof(vs[0]); ++v) {
    if (skip(vs[v].name)) continue;
    CHECK(hipMemset(C, 0, (size_t)M * N * 2));
    CHECK(hipMemset(err, 0, 4));
    const int gv = vs[v].all_tiles ? (M / 256) * (N / 256) : grid;
    hipLaunchKernelGGL(vs[v].fn, dim3(gv), dim3(vs[v].threads), 0, 0, a);
    CHECK(hipGetLastError());
    cmp_kernel<<<1024, 256>>>(C, R, (size_t)M * N, err);
    float e = 0;
    CHECK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    printf("%-20s max|err| = %.4g %s\n", vs[v].name, e, e < 2e-3 * K ? "ok" : "FAIL");
  }
  for (int r = 0; r < rounds; ++r)
    for (size_t v = 0; v < sizeof(vs) / sizeof(vs[0]); ++v) {
      if (skip(vs[v].name)) continue;
      const int gv = vs[v].all_tiles ? (M / 256) * (N / 256) : grid;
      for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(vs[v].fn, dim3(gv), dim3(vs[v].threads), 0, 0, a);
      CHECK(hipEventRecord(e0));
      for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(vs[v].fn, dim3(gv), dim3(vs[v].threads), 0, 0, a);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      times[v].push_back(ms / iters);
    }
  printf("\n%dx%dx%d bf16, grid %d\n", M, N, K, grid);
  for (size_t v = 0; v < sizeof(vs) / sizeof(vs[0]); ++v) {
    auto t = times[v];
    if (t.empty()) continue;
    std::sort(t.begin(), t.end());
    const float med = t[t.size() / 2];
    printf("  %-20s %8.4f ms  %7.1f TFLOP/s\n", vs[v].name, med, flop / (med * 1e-3) / 1e12);
  }
  if (getenv("LAB_STAMP")) {
    // pt4 (nt stores) with s_memtime buckets: per K-tile cycles per wave, by wave group
    Args s = a;
    s.stamps = stamps;
    for (int i = 0; i < 50; ++i) hipLaunchKernelGGL((pt4_kernel<false, 16>), dim3(grid), dim3(512), 0, 0, a);
    CHECK(hipMemset(stamps, 0, ((size_t)grid * 8 * 16 + 8) * 8));
    if (getenv("LAB_STAMP")[0] == 'b')
      hipLaunchKernelGGL((pt4_kernel<true, 16 | 65536>), dim3(grid), dim3(512), 0, 0, s);
    else if (getenv("LAB_STAMP")[0] == 'v')
      hipLaunchKernelGGL((pt4v_kernel<true, 15>), dim3(grid), dim3(512), 0, 0, s);
    else if (getenv("LAB_STAMP")[0] == 'w')
      hipLaunchKernelGGL((pt4v_kernel<true, 0>), dim3(grid), dim3(512), 0, 0, s);
    else if (getenv("LAB_STAMP")[0] == 'k')
      hipLaunchKernelGGL((pt4k_kernel<true>), dim3(grid), dim3(512), 0, 0, s);
    else if (getenv("LAB_STAMP")[0] == 'x')
      hipLaunchKernelGGL((pt4v_kernel<true, 31>), dim3(grid), dim3(512), 0, 0, s);
    else
      hipLaunchKernelGGL((pt4_kernel<true, 16>), dim3(grid), dim3(512), 0, 0, s);
    CHECK(hipDeviceSynchronize());
    std::vector<unsigned long long> h((size_t)grid * 8 * 16);
    CHECK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
    const char* names[15] = {"A:ds_read issue", "A:glds issue", "A:lgkm wait", "B:ds_read issue",
                             "B:glds issue", "B:lgkm wait", "vm waits", "bar after load A",
                             "bar after mfma A", "bar after load B", "bar after mfma B",
                             "mfma A issue", "mfma B issue", "C stores", "total"};
    for (int g = 0; g < 2; ++g) {
      double sum[15] = {}, kt = 0;
      for (int b = 0; b < grid; ++b)
        for (int w = g * 4; w < g * 4 + 4; ++w) {
          const unsigned long long* o = &h[((size_t)b * 8 + w) * 16];
          for (int j = 0; j < 15; ++j) sum[j] += (double)o[j];
          kt += (double)o[15] * (K / 64);
        }
      printf("pt4 stamps, waves %d-%d, cycles per K-tile per wave:\n", g * 4, g * 4 + 3);
      for (int j = 0; j < 15; ++j) printf("    %-18s %6.0f\n", names[j], sum[j] / kt);
    }
    printf("ideal: 4 x 32 MFMA x 16 cyc = 2048 per K-tile per SIMD (1024 issue per wave)\n");
  }
  return 0;
}
