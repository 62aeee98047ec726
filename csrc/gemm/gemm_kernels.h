// CDNA4 (gfx950) MFMA GEMM kernels and their launch templates (device code, header-only).
// Included by one translation unit per input dtype (gemm_<dtype>.hip) so the kernels compile in
// parallel; the public entry points live in gemm_mfma.hip. Design notes: gemm_mfma.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include <type_traits>

#include "gemm.h"
#include "tile_map.h"

namespace ddlb {
namespace {

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;

#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))

__device__ __forceinline__ void glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds((const GLB_AS void*)g, (LDS_AS void*)lds, 16, 0, 0);
}

// Address of logical A row ``row``: grouped rows, or a per-shard pointer table (direct access).
__device__ __forceinline__ const char* a_row(const GemmArgs& p, int64_t row, int esz) {
  if (p.a_table != nullptr) {
    const unsigned ur = (unsigned)row, us = (unsigned)p.shard_rows;
    const unsigned sh = ur / us;
    return (const char*)p.a_table[sh] + (int64_t)(ur - sh * us) * p.lda * esz;
  }
  return (const char*)p.a + map_row(row, p.a_grp, p.a_gstride) * p.lda * esz;
}

// Address of logical C row ``row``: grouped rows, or a per-shard pointer table (direct store:
// row block s of c_shard_rows rows lives at c_table[s], e.g. a peer's receive slot over xGMI).
// DS: 0 = grouped rows only (no table), 1 = table only, 2 = decided at run time. The persistent
// pt4 kernel (the flagship's) is instantiated per form: the run-time branch in its epilogue cost
// ~8 % (profiles/r02/s4/r2s4_7_*). Both forms are built as global-address-space pointers: a
// pointer read from the table is otherwise "generic", and the merged value would turn every
// epilogue store into a flat store.
template <int OSZ, int DS = 2>
__device__ __forceinline__ char* c_row(const GemmArgs& p, int64_t row) {
  if constexpr (DS == 0) return (char*)p.c + map_row(row, p.c_grp, p.c_gstride) * p.ldc * OSZ;
  GLB_AS char* base;
  if (DS == 1 || p.c_table != nullptr) {
    const unsigned ur = (unsigned)row, us = (unsigned)p.c_shard_rows;
    const unsigned sh = ur / us;
    base = (GLB_AS char*)p.c_table[sh] + (int64_t)(ur - sh * us) * p.ldc * OSZ;
  } else {
    base = (GLB_AS char*)p.c + map_row(row, p.c_grp, p.c_gstride) * p.ldc * OSZ;
  }
  return (char*)base;
}

__device__ __forceinline__ int tile_index(const GemmArgs& p, int nwg) {
  return tile_index_virtual(p, (int)blockIdx.x, nwg);
}

// ---------------------------------------------------------------- MFMA "consume 16 bytes" ops
struct MmaBF16 {
  static constexpr int kElem = 2, kMfma = 1;  // bytes per element, MFMAs per 16-byte step
  static __device__ __forceinline__ void step(f32x4& acc, const i32x4& b, const i32x4& a) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, b),
                                                  __builtin_bit_cast(bf16x8, a), acc, 0, 0, 0);
  }
};
struct MmaF16 {
  static constexpr int kElem = 2, kMfma = 1;
  static __device__ __forceinline__ void step(f32x4& acc, const i32x4& b, const i32x4& a) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, b),
                                                 __builtin_bit_cast(f16x8, a), acc, 0, 0, 0);
  }
};
struct MmaFP8 {  // OCP e4m3 x e4m3, f32 accumulate; 2 instructions per 16 B
  static constexpr int kElem = 1, kMfma = 2;
  static __device__ __forceinline__ void step(f32x4& acc, const i32x4& b, const i32x4& a) {
    const long b0 = ((long)(unsigned)b.y << 32) | (unsigned)b.x;
    const long b1 = ((long)(unsigned)b.w << 32) | (unsigned)b.z;
    const long a0 = ((long)(unsigned)a.y << 32) | (unsigned)a.x;
    const long a1 = ((long)(unsigned)a.w << 32) | (unsigned)a.z;
    acc = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(b0, a0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(b1, a1, acc, 0, 0, 0);
  }
};
struct MmaF32 {  // exact f32 MFMA; 4 instructions per 16 B
  static constexpr int kElem = 4, kMfma = 4;
  static __device__ __forceinline__ void step(f32x4& acc, const i32x4& b, const i32x4& a) {
    const f32x4 bf = __builtin_bit_cast(f32x4, b), af = __builtin_bit_cast(f32x4, a);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(bf.x, af.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(bf.y, af.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(bf.z, af.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(bf.w, af.w, acc, 0, 0, 0);
  }
};

// Block-scaled MX-fp8 (e4m3 x e4m3, unit E8M0 scales = 127): ONE v_mfma_scale_f32_16x16x128_f8f6f4
// consumes both 16-byte chunks of a 128-byte K-row (kPair), at 2x the bf16 MFMA rate.
struct MmaMX {
  static constexpr int kElem = 1, kMfma = 1;
  static constexpr bool kPair = true;
  static __device__ __forceinline__ void step8(f32x4& acc, const i32x8& b, const i32x8& a) {
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b, a, acc, 0, 0, 0, 127, 0, 127);
  }
};
template <class Mma, class = void> struct is_pair : std::false_type {};
template <class Mma> struct is_pair<Mma, std::void_t<decltype(Mma::kPair)>>
    : std::integral_constant<bool, Mma::kPair> {};

// Compile-time emission of the {PER x MFMA, 1 x VMEM, n_g x DS_READ} interleave pattern
// (sched_group_barrier arguments must be literal constants).
template <int G, int NG, int PER, int NRD, int NDMA>
struct IlvPattern {
  static __device__ __forceinline__ void emit() {
    if constexpr (G < NG) {
      __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      constexpr int nrd = ((G + 1) * NRD) / NDMA - (G * NRD) / NDMA;
      if constexpr (nrd > 0) __builtin_amdgcn_sched_group_barrier(0x100, nrd, 0);
      IlvPattern<G + 1, NG, PER, NRD, NDMA>::emit();
    }
  }
};

// ---------------------------------------------------------------- fused epilogue activation
__device__ __forceinline__ float act1(float x, int act) {
  switch (act) {
    case ACT_GELU: {  // tanh approximation (what Megatron / TE use for GPT-style MLPs)
      const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
      return 0.5f * x * (1.f + tanhf(u));
    }
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_SILU: return x / (1.f + __expf(-x));
    default: return x;
  }
}
__device__ __forceinline__ f32x4 act4(f32x4 v, int act) {
  if (act == ACT_NONE) return v;
  return f32x4{act1(v.x, act), act1(v.y, act), act1(v.z, act), act1(v.w, act)};
}

// ---------------------------------------------------------------- output conversion
template <int OUT> struct Store4;
template <> struct Store4<DT_BF16> {
  static __device__ __forceinline__ void st(void* p, const f32x4 v) {
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    bf16x4 o = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    *(uint2*)p = __builtin_bit_cast(uint2, o);
  }
  static __device__ __forceinline__ void st1(void* p, float v) { *(__bf16*)p = (__bf16)v; }
};
template <> struct Store4<DT_F16> {
  static __device__ __forceinline__ void st(void* p, const f32x4 v) {
    typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
    f16x4 o = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
    *(uint2*)p = __builtin_bit_cast(uint2, o);
  }
  static __device__ __forceinline__ void st1(void* p, float v) { *(_Float16*)p = (_Float16)v; }
};
template <> struct Store4<DT_F32> {
  static __device__ __forceinline__ void st(void* p, const f32x4 v) { *(f32x4*)p = v; }
  static __device__ __forceinline__ void st1(void* p, float v) { *(float*)p = v; }
};

template <int OUT> constexpr int out_size() { return OUT == DT_F32 ? 4 : 2; }

// ---------------------------------------------------------------- bounded arrival spin
// A tile reads the physical A rows map_row(m0) .. map_row(last row of the tile), which can span
// several shards when the shard height (flag_rows) is not a multiple of the tile height (e.g.
// m/d = 320 rows with 128- or 256-row tiles): wait for EVERY shard in that range, not only the
// first row's. The acquire is at system scope: the rows were written by a copy engine or by a
// peer GPU over xGMI, not by this agent.
// Thread 0 spins and acquires; the caller orders the other threads after it with a barrier.
template <bool OWN_FIRST = true>  // false: tile_order 3 compiled out (see tile_map.h)
__device__ __forceinline__ void wait_flag_t0(const GemmArgs& p, int64_t row_first,
                                             int64_t row_last) {
  if (threadIdx.x == 0) {
    const int s0 = (int)(row_first / p.flag_rows), s1 = (int)(row_last / p.flag_rows);
    const unsigned want = p.epoch_ptr ? *p.epoch_ptr : p.epoch;
    for (int sh = s0; sh <= s1; ++sh) {
      // tile_order 3: the first producer's blocks are the caller's own rows (never gated)
      if (OWN_FIRST && p.tile_order == 3 && sh / p.nsub == p.first_shard) continue;
      unsigned* f = const_cast<unsigned*>(p.flags) + sh;
      unsigned spins = 0;
      while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > p.spin_limit) {  // give up, report, let the grid drain
          if (p.timeout_word) atomicOr(p.timeout_word, 1u);
          break;
        }
      }
    }
    // system scope: the rows were written by a copy engine or a peer GPU. When only this
    // launch's own copy workgroups set the flags (in-kernel all-gather, AG_AGENT_ACQUIRE) an
    // agent-scope acquire covers them (write-through stores, MI355X guide §6 Guideline 16 R1).
    if (p.ag_mode & AG_AGENT_ACQUIRE)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    else
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
}

template <bool OWN_FIRST = true>
__device__ __forceinline__ void wait_flag(const GemmArgs& p, int64_t row_first, int64_t row_last) {
  if (p.flags == nullptr) return;
  wait_flag_t0<OWN_FIRST>(p, row_first, row_last);
  __syncthreads();
}

// ---------------------------------------------------------------- in-kernel all-gather
// The copy workgroups of a flag-gated pt4 launch (GemmArgs::ag_ctas). Work units are
// (block, part, producer), block-major with producers in ring order from rank + 1 innermost: the
// block order the gated GEMM dispatches its tiles in (ordered_shard), all links busy at once.
// Each unit is a contiguous byte range of the same rows in the producer's A and ours; U x 16-byte
// loads in flight per thread.
// Publication (default, MI355X guide §6 Guideline 16 R1): the payload is stored WRITE-THROUGH
// (16-byte `sc1` buffer stores), every wave drains its stores (vmcnt(0)), a workgroup barrier,
// then thread 0 counts the unit with a relaxed agent atomic; the last part of a segment sets its
// flag (atomic store), the last unit of a producer ACKs it over xGMI. No release fence: an
// agent-scope release is a `buffer_wbl2` of the whole XCD L2, dirty C tiles of the GEMM
// workgroups on that XCD included, once per unit. AG_LEGACY_PUBLISH keeps the plain-store +
// release-fence form for comparison (scripts/bench_agk_world1.py).
typedef __attribute__((ext_vector_type(4))) unsigned ag_u32x4;
template <int U, bool WT>
__device__ __forceinline__ void ag_copy_bytes(const GLB_AS ag_u32x4* src, char* dst, int64_t nvec,
                                              int tid) {
  constexpr int T = 512;
  // wave-uniform descriptor over this unit (a unit is < 1 GiB, checked at launch)
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)dst, 0, (int)(nvec * 16), 0x00020000);
  GLB_AS ag_u32x4* d = (GLB_AS ag_u32x4*)dst;
  auto st = [&](int64_t v, ag_u32x4 x) __attribute__((always_inline)) {
    if constexpr (WT)
      __builtin_amdgcn_raw_buffer_store_b128(x, r, (unsigned)(v * 16), 0, 16 /* sc1 */);
    else
      d[v] = x;
  };
  int64_t v = tid;
  for (; v + (U - 1) * T < nvec; v += U * T) {
    ag_u32x4 x[U];
#pragma unroll
    for (int i = 0; i < U; ++i) x[i] = src[v + i * T];
#pragma unroll
    for (int i = 0; i < U; ++i) st(v + i * T, x[i]);
  }
  for (; v < nvec; v += T) st(v, src[v]);
}

template <int ESZ>
__device__ __forceinline__ void ag_copy_role(const GemmArgs& p) {
  const unsigned want = p.epoch_ptr ? *p.epoch_ptr : p.epoch;
  const int np = p.nshards / p.nsub, s = p.nsub, parts = p.ag_parts;
  const uint64_t* tab = p.ag_tab;
  // every shared word is a GLOBAL (never flat) access
  const GLB_AS unsigned* ready = (const GLB_AS unsigned*)tab[2 * np];
  GLB_AS unsigned* count = (GLB_AS unsigned*)tab[2 * np + 1];
  GLB_AS unsigned* arrive = (GLB_AS unsigned*)p.flags;
  const int64_t seg = p.flag_rows * p.lda * ESZ;
  const int64_t part = (seg / parts + 15) / 16 * 16;
  const int per_b = (np - 1) * parts, units = s * per_b;
  const int tid = threadIdx.x;
  const bool legacy = (p.ag_mode & AG_LEGACY_PUBLISH) != 0;
  const bool deep = (p.ag_mode & AG_DEEP_LOADS) != 0;
  unsigned seen = 0;
  for (int u = (int)blockIdx.x; u < units; u += p.ag_ctas) {
    int b, prod, pi;  // every peer's units interleaved (tile_map.h)
    ag_unit(u, np, parts, p.ag_rank, b, prod, pi);
    if (!((seen >> prod) & 1u)) {  // first unit of this producer: its READY, acquired
      if (tid == 0) {
        unsigned spins = 0;
        while (__hip_atomic_load(ready + prod, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) <
               want) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > p.spin_limit) {
            if (p.timeout_word) atomicOr(p.timeout_word, 4u);
            break;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
      }
      __syncthreads();
      seen |= 1u << prod;
    }
    const int64_t base = (int64_t)(prod * s + b) * seg + (int64_t)pi * part;
    int64_t nb = seg - (int64_t)pi * part;
    nb = nb < part ? nb : part;
    const GLB_AS ag_u32x4* src = (const GLB_AS ag_u32x4*)(tab[prod] + base);
    char* dst = (char*)p.a + base;
    const int64_t nvec = nb > 0 ? nb / 16 : 0;
    if (legacy) {
      ag_copy_bytes<8, false>(src, dst, nvec, tid);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    } else {
      if (deep)
        ag_copy_bytes<16, true>(src, dst, nvec, tid);
      else
        ag_copy_bytes<8, true>(src, dst, nvec, tid);
      // every wave drains its write-through stores (and its peer loads) before the count
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (tid == 0) {
      const int sh = prod * s + b;
      if (__hip_atomic_fetch_add(count + sh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 ==
          want * (unsigned)parts)
        __hip_atomic_store(arrive + sh, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // ACK: every load of the producer's rows by this unit has returned (vmcnt(0) / the
      // release above), so a relaxed store suffices; it crosses xGMI, hence system scope
      if (__hip_atomic_fetch_add(count + np * s + prod, 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT) + 1 == want * (unsigned)(s * parts))
        __hip_atomic_store((GLB_AS unsigned*)tab[np + prod], want, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if ((p.ag_mode & AG_WAIT_ACKS) && blockIdx.x == 0 && tid == 0) {
    // every peer has finished reading my rows before the launch ends (the caller may then
    // overwrite them): the plan's ACK wait, without a kernel of its own after this one
    for (int q = 0; q < np; ++q) {
      if (q == p.ag_rank) continue;
      const GLB_AS unsigned* a = (const GLB_AS unsigned*)tab[2 * np + 2 + q];
      unsigned spins = 0;
      while (__hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > p.spin_limit) {
          if (p.timeout_word) atomicOr(p.timeout_word, 8u);
          break;
        }
      }
    }
  }
}

// Arrival wait for the tile whose first logical row is m0 and which has (up to) BM rows.
__device__ __forceinline__ void wait_tile(const GemmArgs& p, int64_t m0, int BM) {
  if (p.flags == nullptr) return;
  const int64_t last = (m0 + BM < p.M ? m0 + BM : p.M) - 1;
  wait_flag(p, map_row(m0, p.a_grp, p.a_gstride), map_row(last, p.a_grp, p.a_gstride));
}

// ---------------------------------------------------------------- the tiled kernel
template <class Mma, int OUT, int BM, int BN, int WM, int WN, bool ILV = false>
__global__ __launch_bounds__(WM* WN * 64) void gemm_tn_kernel(const GemmArgs p) {
  constexpr int NT = WM * WN * 64, NW = WM * WN;
  constexpr int ROWB = 128;  // bytes per row per K-tile
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE = A_BYTES + B_BYTES;
  constexpr int TM = BM / WM, TN = BN / WN, MR = TM / 16, NR = TN / 16;
  constexpr int LA = BM / 8 / NW, LB = BN / 8 / NW;  // LDS-DMA instructions per wave per tile
  static_assert(LA * NW * 8 == BM && LB * NW * 8 == BN, "tile rows must split over waves");
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int wg = tile_index(p, nwg);
  const int tm = wg / tiles_n, tn = wg % tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

  // Per-lane source pointers for the LDS-DMA rows this wave stages.
  const int esz = Mma::kElem;
  const char* aptr[LA];
  const char* bptr[LB];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    const int row = (wave * LA + i) * 8 + (lane >> 3);
    int64_t gr = m0 + row;
    gr = gr < p.M ? gr : p.M - 1;
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    aptr[i] = a_row(p, gr, esz) + chunk * 16;
  }
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int row = (wave * LB + i) * 8 + (lane >> 3);
    int64_t gr = n0 + row;
    gr = gr < p.N ? gr : p.N - 1;
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    bptr[i] = (const char*)p.b + gr * p.ldb * esz + chunk * 16;
  }

  wait_tile(p, m0, BM);

  auto stage = [&](int buf, int kt) __attribute__((always_inline)) {
    char* base = smem + buf * STAGE;
    const int64_t koff = (int64_t)kt * ROWB;
#pragma unroll
    for (int i = 0; i < LA; ++i) glds16(aptr[i] + koff, base + (wave * LA + i) * 1024);
#pragma unroll
    for (int i = 0; i < LB; ++i) glds16(bptr[i] + koff, base + A_BYTES + (wave * LB + i) * 1024);
  };

  const int wm = wave / WN, wn = wave % WN;
  const int swz = (lane & 15) >> 1;
  const int frow = lane & 15, fq = lane >> 4;
  f32x4 acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) __attribute__((always_inline)) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int c4 = 0; c4 < 8; c4 += 4) {
      const int choff = ((c4 + fq) ^ swz) * 16;
      i32x4 af[MR], bfr[NR];
#pragma unroll
      for (int i = 0; i < MR; ++i)
        af[i] = *(const i32x4*)(As + (wm * TM + i * 16 + frow) * ROWB + choff);
#pragma unroll
      for (int j = 0; j < NR; ++j)
        bfr[j] = *(const i32x4*)(Bs + (wn * TN + j * 16 + frow) * ROWB + choff);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j) Mma::step(acc[i][j], bfr[j], af[i]);
      __builtin_amdgcn_s_setprio(0);
    }
  };

  // Interleaved variant: the next tile's LDS-DMA is issued INSIDE the first MFMA cluster (one
  // DMA per MR*NR/(LA+LB) MFMAs), so its issue cost hides behind the matrix pipe instead of
  // forming a burst at the top of every K-tile (cdna guide: "the per-phase interleave is the
  // lever"). The DMA writes the other LDS buffer, so it may be placed after this tile's reads.
  auto compute_ilv = [&](int buf, int next_kt) __attribute__((always_inline)) {
    // First half: MFMAs on the c4=0 fragments, with the next tile's LDS-DMA (1 per PER MFMAs)
    // and the c4=4 fragment reads (into a second register set) interleaved between them.
    constexpr int NDMA = LA + LB, NRD = MR + NR, NQ = MR * NR;
    constexpr int PER = NQ / NDMA > 0 ? NQ / NDMA : 1;
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES;
    char* nbase = smem + (buf ^ 1) * STAGE;
    const int64_t koff = (int64_t)next_kt * ROWB;
    const int ch0 = ((0 + fq) ^ swz) * 16, ch1 = ((4 + fq) ^ swz) * 16;
    i32x4 af0[MR], bf0[NR], af1[MR], bf1[NR];
#pragma unroll
    for (int i = 0; i < MR; ++i)
      af0[i] = *(const i32x4*)(As + (wm * TM + i * 16 + frow) * ROWB + ch0);
#pragma unroll
    for (int j = 0; j < NR; ++j)
      bf0[j] = *(const i32x4*)(Bs + (wn * TN + j * 16 + frow) * ROWB + ch0);
    auto rd1 = [&](int r) __attribute__((always_inline)) {
      if (r < MR) af1[r] = *(const i32x4*)(As + (wm * TM + r * 16 + frow) * ROWB + ch1);
      else bf1[r - MR] = *(const i32x4*)(Bs + (wn * TN + (r - MR) * 16 + frow) * ROWB + ch1);
    };
    auto dma = [&](int d) __attribute__((always_inline)) {
      if (d < LA) glds16(aptr[d] + koff, nbase + (wave * LA + d) * 1024);
      else glds16(bptr[d - LA] + koff, nbase + A_BYTES + (wave * LB + d - LA) * 1024);
    };
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      Mma::step(acc[q / NR][q % NR], bf0[q % NR], af0[q / NR]);
      if ((q % PER) == PER - 1) {
        const int g = q / PER;
        if (g < NDMA) dma(g);
        // spread the NRD second-half reads over the NDMA groups
#pragma unroll
        for (int r = (g * NRD) / NDMA; r < ((g + 1) * NRD) / NDMA; ++r) rd1(r);
      }
    }
#pragma unroll
    for (int d = NQ / PER; d < NDMA; ++d) dma(d);
#pragma unroll
    for (int r = ((NQ / PER) * NRD) / NDMA; r < NRD; ++r) rd1(r);
    IlvPattern<0, (NDMA < NQ / PER ? NDMA : NQ / PER), PER, NRD, NDMA>::emit();
#pragma unroll
    for (int q = 0; q < NQ; ++q) Mma::step(acc[q / NR][q % NR], bf1[q % NR], af1[q / NR]);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = p.K * esz / ROWB;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  int cur = 0;
  for (int kt = 0; kt < nk - 1; ++kt) {
    if constexpr (ILV) {
      compute_ilv(cur, kt + 1);
    } else {
      stage(cur ^ 1, kt + 1);
      compute(cur);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur ^= 1;
  }
  compute(cur);

  // Epilogue: lane holds C[row = .. + frow][col = .. + 4*fq + r], r = 0..3.
  constexpr int OSZ = out_size<OUT>();
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    const int64_t row = m0 + wm * TM + i * 16 + frow;
    if (row >= p.M) continue;
    char* crow = c_row<OSZ>(p, row);
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int64_t col = n0 + wn * TN + j * 16 + fq * 4;
      if (col + 3 < p.N) {
        Store4<OUT>::st(crow + col * OSZ, act4(acc[i][j], p.act));
      } else {
        const f32x4 a4 = act4(acc[i][j], p.act);
        const float v[4] = {a4.x, a4.y, a4.z, a4.w};
        for (int r = 0; r < 4; ++r)
          if (col + r < p.N) Store4<OUT>::st1(crow + (col + r) * OSZ, v[r]);
      }
    }
  }
}

// ---------------------------------------------------------------- counted waits, C stores
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 8 consecutive outputs from two f32x4, written with non-temporal (streaming) stores: C is not
// re-read by the kernel, and keeping 128 MB of output lines out of the L2 allocation leaves it
// to the A / B panels (lab, profiles/r01/s2/lab/pt4_nt_*: flagship pt4 0.1126 -> 0.1063 ms,
// 8192^3 0.817 -> 0.806 ms).
template <int OUT> struct Store8;
template <> struct Store8<DT_BF16> {
  static constexpr int kStores = 1;
  static __device__ __forceinline__ void st(void* p, const f32x4 a, const f32x4 b) {
    bf16x8 o = {(__bf16)a.x, (__bf16)a.y, (__bf16)a.z, (__bf16)a.w,
                (__bf16)b.x, (__bf16)b.y, (__bf16)b.z, (__bf16)b.w};
    __builtin_nontemporal_store(__builtin_bit_cast(i32x4, o), (i32x4*)p);
  }
};
template <> struct Store8<DT_F16> {
  static constexpr int kStores = 1;
  static __device__ __forceinline__ void st(void* p, const f32x4 a, const f32x4 b) {
    f16x8 o = {(_Float16)a.x, (_Float16)a.y, (_Float16)a.z, (_Float16)a.w,
               (_Float16)b.x, (_Float16)b.y, (_Float16)b.z, (_Float16)b.w};
    __builtin_nontemporal_store(__builtin_bit_cast(i32x4, o), (i32x4*)p);
  }
};
template <> struct Store8<DT_F32> {
  static constexpr int kStores = 2;
  static __device__ __forceinline__ void st(void* p, const f32x4 a, const f32x4 b) {
    __builtin_nontemporal_store(a, (f32x4*)p);
    __builtin_nontemporal_store(b, (f32x4*)p + 1);
  }
};

// The same 8 outputs through a buffer descriptor over C with cache bits sc1 | nt (aux 18): the
// line leaves this XCD's L2 as it is written (write-through) instead of staying there as a dirty
// streaming line. GEMM lab, one box (profiles/r02/s4/r2s4_17_*): pt4 flagship 0.1060 -> 0.1040 ms,
// 16384x8192x1024 0.2347 -> 0.2177 ms vs plain nt stores.
// soff: a wave-uniform part of the offset (SGPR soffset), so a kernel can keep the per-lane part
// fixed and move only scalars per store (pt4).
// (AUX 18 = sc1 | nt; 16 = sc1 alone, the K-split hand-off. For the C tiles, r5_6 measured nt
// alone equal to sc1 | nt and sc1 alone 2.5-12 % slower: flagship 0.1118 / 0.1111 / 0.1249 ms)
// 8 outputs (two f32x4) rounded to the 16-bit C type, as the 16 bytes one lane stores
template <int OUT>
__device__ __forceinline__ __attribute__((ext_vector_type(4))) unsigned pack8(const f32x4 a,
                                                                             const f32x4 b) {
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
  static_assert(OUT == DT_BF16 || OUT == DT_F16, "16-bit outputs only");
  if constexpr (OUT == DT_BF16) {
    const bf16x8 o = {(__bf16)a.x, (__bf16)a.y, (__bf16)a.z, (__bf16)a.w,
                      (__bf16)b.x, (__bf16)b.y, (__bf16)b.z, (__bf16)b.w};
    return __builtin_bit_cast(u32x4_t, o);
  } else {
    const f16x8 o = {(_Float16)a.x, (_Float16)a.y, (_Float16)a.z, (_Float16)a.w,
                     (_Float16)b.x, (_Float16)b.y, (_Float16)b.z, (_Float16)b.w};
    return __builtin_bit_cast(u32x4_t, o);
  }
}

// f32 (SWZ, the pt4 fragment layout: lane group g = lane >> 4 holds columns 8g .. 8g+7 of a
// 32-column quadrant, `off` = its own 8 columns): storing a | b as they are makes each
// instruction write 16 of every 32 bytes of the quadrant's rows, and write-through stores then
// reach HBM as half-filled sectors (f32 K-split partials measured 2x slower than bf16 ones,
// r5_12). One v_permlane32_swap per dword (lanes 32-63 of a <-> lanes 0-31 of b) regroups them:
// a then holds columns {0-3, 8-11, 4-7, 12-15} in groups 0..3 and b the same + 16, so each
// instruction writes 64 contiguous bytes per row (cdna guide T21). Needs all 64 lanes active.
template <int OUT, int AUX = 18, bool SWZ = true>
__device__ __forceinline__ void store8_wt(__amdgpu_buffer_rsrc_t rc, unsigned off, const f32x4 a,
                                          const f32x4 b, unsigned soff = 0) {
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
  if constexpr (OUT == DT_F32 && SWZ) {
    u32x4_t x = __builtin_bit_cast(u32x4_t, a), y = __builtin_bit_cast(u32x4_t, b);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const auto r = __builtin_amdgcn_permlane32_swap(x[i], y[i], false, false);
      x[i] = r[0];
      y[i] = r[1];
    }
    // groups 2, 3 now store columns 4-7 / 12-15 (x) of the quadrant: 12 columns left of their own
    const unsigned o = (__lane_id() & 32) ? off - 48 : off;
    __builtin_amdgcn_raw_buffer_store_b128(x, rc, o, soff, AUX);
    __builtin_amdgcn_raw_buffer_store_b128(y, rc, o + 64, soff, AUX);
  } else if constexpr (OUT == DT_F32) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, a), rc, off, soff, AUX);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, b), rc, off + 16, soff, AUX);
  } else if constexpr (OUT == DT_BF16) {
    bf16x8 o = {(__bf16)a.x, (__bf16)a.y, (__bf16)a.z, (__bf16)a.w,
                (__bf16)b.x, (__bf16)b.y, (__bf16)b.z, (__bf16)b.w};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), rc, off, soff, AUX);
  } else {
    f16x8 o = {(_Float16)a.x, (_Float16)a.y, (_Float16)a.z, (_Float16)a.w,
               (_Float16)b.x, (_Float16)b.y, (_Float16)b.z, (_Float16)b.w};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, o), rc, off, soff, AUX);
  }
}

// ---------------------------------------------------------------- t8: 8-phase ping-pong kernel
// 256x256 tile, BK = one 128-byte row (64 bf16 / 128 fp8 / 32 f32), 8 waves = 2 groups (wr) x 4
// (wc), 128x64 per wave as 2x2 quadrants of 64x32 (cdna guide §5 "256^2 8-phase template",
// T2+T3+T4+T5). Group 1 runs one barrier behind group 0, so between any two barriers one group
// issues ds_reads + LDS-DMA while the other runs 16 MFMAs. K-tile data moves in 16 KB units of
// 128 rows: UA0 = A rows {0-63, 128-191} (quadrant row mq=0 of both groups), UA1 = {64-127,
// 192-255}, UB0 = B rows {wc*64 + 0..31}, UB1 = {wc*64 + 32..63}; wave w stages unit rows
// [16w, 16w+16) (2 x 1 KB LDS-DMA). K-tile t lives in buffer t&1; phase p of a group
// (intervals I_k between barriers, group g reads in I_{8t+2p+g}):
//   p0: read A(mq0) + B(nq0), stage UA1(t+1)   p1: read B(nq1), stage UB0(t+1)
//   p2: read A(mq1),          stage UA0(t+2)   p3: read B(nq0), stage UB1(t+2), vmcnt(4)
// RAW: vmcnt(4) (2 unit slices in flight) before barrier 8(t+1) retires every slice of K-tile t+1
// on every wave (group 1 in its p3 read section, group 0 after its p3 MFMAs).
// WAR: each unit is restaged 3 intervals after its last read (reads retire by lgkmcnt(0) in the
// next interval), e.g. UA0 of t is read in I_{8t}, I_{8t+1} and restaged in I_{8t+4}, I_{8t+5}.
// Past the last K-tile the stage source is clamped to K-tile nk-1: identical bytes into units no
// one reads again, so the vmcnt arithmetic stays uniform. B rows are loaded permuted within each
// 32-row quadrant so a lane's two fragments of a quadrant hold 8 consecutive output columns (one
// 16-byte store). Measured (profiles/r01/s2/lab/t8_vs_ring2.txt): 1425 TF at 8192^3 (+55 % over
// the ring kernel, within 2 % of hipBLASLt), +7 % on the 65536x1024x1024 flagship.
__device__ __forceinline__ int t8_perm(int t) { return 8 * ((t & 15) >> 2) + 4 * (t >> 4) + (t & 3); }

template <class Mma, int OUT>
__global__ __launch_bounds__(512) void gemm_tn_t8_kernel(const GemmArgs p) {
  constexpr int ROWB = 128, UNIT = 128 * ROWB, STAGE = 4 * UNIT;
  constexpr int UA0 = 0, UA1 = UNIT, UB0 = 2 * UNIT, UB1 = 3 * UNIT;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int wg = tile_index(p, ntiles);
  int tm_, tn_;
  tile_mn(p, wg, p.M / 256, tiles_n, tm_, tn_);
  const int64_t m0 = (int64_t)tm_ * 256, n0 = (int64_t)tn_ * 256;
  const int esz = Mma::kElem;
  const int nk = p.K * esz / ROWB;

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
      sA[q][i] = a_row(p, m0 + lr, esz) + ch;
      const int lc = (ur >> 5) * 64 + q * 32 + t8_perm(ur & 31);
      sB[q][i] = (const char*)p.b + (n0 + lc) * p.ldb * esz + ch;
    }
  }
  wait_tile(p, m0, 256);
  auto stage = [&](const char* const* src, int unit_off, int kt, int buf) __attribute__((always_inline)) {
    kt = kt < nk ? kt : nk - 1;
    char* dst = smem + buf * STAGE + unit_off + wave * 16 * ROWB;
    glds16(src[0] + (int64_t)kt * ROWB, dst);
    glds16(src[1] + (int64_t)kt * ROWB, dst + 8 * ROWB);
  };

  // ---- fragment reads: unit row base + (lane & 15), logical chunk kk*4 + (lane >> 4)
  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;
  const int c0 = ((0 + fq) ^ sw) * 16, c1 = ((4 + fq) ^ sw) * 16;
  const int aoff = (wr * 64 + frow) * ROWB, boff = (wc * 32 + frow) * ROWB;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x4 aR[4][2], bR[2][2];  // fragments: [f or g][K-half]
  i32x8 aP[4], bP[2];        // MX (kPair): both K-halves in one register tuple, loaded in place
  constexpr bool PAIR = is_pair<Mma>::value;
  auto loadA = [&](const char* base, int mq) __attribute__((always_inline)) {
    const char* r = base + (mq ? UA1 : UA0) + aoff;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      if constexpr (PAIR) {
        aP[f].lo = *(const i32x4*)(r + f * 16 * ROWB + c0);
        aP[f].hi = *(const i32x4*)(r + f * 16 * ROWB + c1);
      } else {
        aR[f][0] = *(const i32x4*)(r + f * 16 * ROWB + c0);
        aR[f][1] = *(const i32x4*)(r + f * 16 * ROWB + c1);
      }
    }
  };
  auto loadB = [&](const char* base, int nq) __attribute__((always_inline)) {
    const char* r = base + (nq ? UB1 : UB0) + boff;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if constexpr (PAIR) {
        bP[g].lo = *(const i32x4*)(r + g * 16 * ROWB + c0);
        bP[g].hi = *(const i32x4*)(r + g * 16 * ROWB + c1);
      } else {
        bR[g][0] = *(const i32x4*)(r + g * 16 * ROWB + c0);
        bR[g][1] = *(const i32x4*)(r + g * 16 * ROWB + c1);
      }
    }
  };
  auto comp = [&](int mq, int nq) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    if constexpr (PAIR) {  // one MFMA per 128-byte K-row
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g) Mma::step8(acc[mq * 4 + f][nq * 2 + g], bP[g], aP[f]);
      // The scaled MFMA is a pure intrinsic: without a use here LLVM sinks all four phases' MFMAs
      // past the barriers to the end of the K-tile (observed: 32 back-to-back MFMAs, spills and
      // vmcnt(0) drains in the loop). An empty asm that "modifies" the quadrant's accumulators
      // pins them inside this phase's compute section.
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g) asm volatile("" : "+v"(acc[mq * 4 + f][nq * 2 + g]));
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
          for (int g = 0; g < 2; ++g) Mma::step(acc[mq * 4 + f][nq * 2 + g], bR[g][kk], aR[f][kk]);
    }
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
  const bool g1 = wr == 1;  // wave-uniform (wave came through readfirstlane)
  if (g1) T8_BAR();
  for (int t = 0; t < nk; ++t) {
    const int b = t & 1, nb = b ^ 1;
    const char* cur = smem + b * STAGE;
    loadA(cur, 0);  // p0
    loadB(cur, 0);
    stage(sA[1], UA1, t + 1, nb);
    T8_BAR();
    comp(0, 0);
    T8_BAR();
    loadB(cur, 1);  // p1
    stage(sB[0], UB0, t + 1, nb);
    T8_BAR();
    comp(0, 1);
    T8_BAR();
    loadA(cur, 1);  // p2
    stage(sA[0], UA0, t + 2, b);
    T8_BAR();
    comp(1, 1);
    T8_BAR();
    loadB(cur, 0);  // p3
    stage(sB[1], UB1, t + 2, b);
    if (g1) wait_vm<4>();
    T8_BAR();
    comp(1, 0);
    if (!g1) wait_vm<4>();
    T8_BAR();
  }
  if (!g1) T8_BAR();
#undef T8_BAR
  wait_vm<0>();  // never leave an LDS-DMA in flight past the end of the workgroup

  // ---- epilogue: a lane holds columns 8*fq .. 8*fq+7 of each 32-column quadrant
  constexpr int OSZ = out_size<OUT>();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t row = m0 + wr * 128 + (i >> 2) * 64 + (i & 3) * 16 + frow;
    char* crow = c_row<OSZ>(p, row);
#pragma unroll
    for (int nq = 0; nq < 2; ++nq) {
      char* dst = crow + (n0 + wc * 64 + nq * 32 + fq * 8) * OSZ;
      // one store site (two branch-local stores get merged by the optimizer, which drops the
      // non-temporal hint)
      f32x4 v0 = acc[i][nq * 2], v1 = acc[i][nq * 2 + 1];
      if (p.act != ACT_NONE) {
        v0 = act4(v0, p.act);
        v1 = act4(v1, p.act);
      }
      Store8<OUT>::st(dst, v0, v1);
    }
  }
}



// ---------------------------------------------------------------- t4: 2-phase ping-pong kernel
// The t8 geometry (256x256 tile, 8 waves in two groups one barrier apart, 16 KB units, 128-byte
// K rows) with 2 phases per K-tile and 32 MFMAs per compute section, i.e. half the barriers:
//   phase A: read A0 + B0 + B1 of K-tile t (16 fragments), stage UA0/UA1(t+1) into the other
//            buffer, compute quadrants (0,0) + (0,1)
//   phase B: read A1 of t (8), stage UB0/UB1(t+2) into this buffer, compute (1,1) + (1,0)
// Every read section ends with lgkmcnt(0) before its barrier, so a unit may be restaged from the
// interval after its last read (UB0/UB1 of t are read only in phase A and held in registers).
// RAW: vmcnt(8) after phase A retires A1 of t (younger: B0/B1(t+1), A0/A1(t+1)); vmcnt(6) after
// phase B retires A0 of t+1, the youngest unit phase A of t+1 reads. Clamped restaging past the
// last K-tile as in t8. Measured (research/lab, profiles/r01/s2/lab/t8_vs_ring2.txt): 9 % faster
// than t8 with one short-K tile per CU (16384x1024x1024), 3 % at 65536x1024x8192, 3 % slower at
// 8192^3.
template <class Mma, int OUT, int CMODE = 0>  // CMODE 2: write-through nt C stores (as pt4)
__global__ __launch_bounds__(512) void gemm_tn_t4_kernel(const GemmArgs p) {
  constexpr int ROWB = 128, UNIT = 128 * ROWB, STAGE = 4 * UNIT;
  constexpr int UA0 = 0, UA1 = UNIT, UB0 = 2 * UNIT, UB1 = 3 * UNIT;
  constexpr bool PAIR = is_pair<Mma>::value;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int wg = tile_index(p, ntiles);
  int tm_, tn_;
  tile_mn(p, wg, p.M / 256, tiles_n, tm_, tn_);
  const int64_t m0 = (int64_t)tm_ * 256, n0 = (int64_t)tn_ * 256;
  const int esz = Mma::kElem;
  const int nk = p.K * esz / ROWB;

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
      sA[q][i] = a_row(p, m0 + lr, esz) + ch;
      const int lc = (ur >> 5) * 64 + q * 32 + t8_perm(ur & 31);
      sB[q][i] = (const char*)p.b + (n0 + lc) * p.ldb * esz + ch;
    }
  }
  wait_tile(p, m0, 256);
  auto stage = [&](const char* const* src, int unit_off, int kt, int buf)
                   __attribute__((always_inline)) {
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
  i32x4 aR[4][2], bR[2][2][2];  // bR[nq][g][K-half]
  i32x8 aP[4], bP[2][2];        // MX (kPair): both K-halves in one register tuple
  auto loadA = [&](const char* base, int mq) __attribute__((always_inline)) {
    const char* r = base + (mq ? UA1 : UA0) + aoff;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      if constexpr (PAIR) {
        aP[f].lo = *(const i32x4*)(r + f * 16 * ROWB + c0);
        aP[f].hi = *(const i32x4*)(r + f * 16 * ROWB + c1);
      } else {
        aR[f][0] = *(const i32x4*)(r + f * 16 * ROWB + c0);
        aR[f][1] = *(const i32x4*)(r + f * 16 * ROWB + c1);
      }
    }
  };
  auto loadB = [&](const char* base, int nq) __attribute__((always_inline)) {
    const char* r = base + (nq ? UB1 : UB0) + boff;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if constexpr (PAIR) {
        bP[nq][g].lo = *(const i32x4*)(r + g * 16 * ROWB + c0);
        bP[nq][g].hi = *(const i32x4*)(r + g * 16 * ROWB + c1);
      } else {
        bR[nq][g][0] = *(const i32x4*)(r + g * 16 * ROWB + c0);
        bR[nq][g][1] = *(const i32x4*)(r + g * 16 * ROWB + c1);
      }
    }
  };
  auto mm = [&](int mq, int nq) __attribute__((always_inline)) {
    if constexpr (PAIR) {
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g) Mma::step8(acc[mq * 4 + f][nq * 2 + g], bP[nq][g], aP[f]);
#pragma unroll
      for (int f = 0; f < 4; ++f)  // pin the pure scaled MFMAs in this section (see t8)
#pragma unroll
        for (int g = 0; g < 2; ++g) asm volatile("" : "+v"(acc[mq * 4 + f][nq * 2 + g]));
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
          for (int g = 0; g < 2; ++g)
            Mma::step(acc[mq * 4 + f][nq * 2 + g], bR[nq][g][kk], aR[f][kk]);
    }
  };
#define T4_BAR()                         \
  do {                                   \
    __builtin_amdgcn_sched_barrier(0);   \
    __builtin_amdgcn_s_barrier();        \
    __builtin_amdgcn_sched_barrier(0);   \
  } while (0)
// compiler-visible lgkmcnt(0) (see pt4)
#define T4_LGKM0()                            \
  do {                                        \
    __builtin_amdgcn_sched_barrier(0);        \
    __builtin_amdgcn_s_waitcnt(0xC07F);       \
    __builtin_amdgcn_sched_barrier(0);        \
  } while (0)
  const bool g1 = wr == 1;  // wave-uniform (wave came through readfirstlane)
  // prologue = the steady-state issue order up to "end of phase B of K-tile -1"
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
    loadB(cur, 0);  // phase A
    loadB(cur, 1);
    loadA(cur, 0);
    stage(sA[0], UA0, t + 1, b ^ 1);
    stage(sA[1], UA1, t + 1, b ^ 1);
    T4_LGKM0();
    if (g1) wait_vm<8>();
    T4_BAR();
    __builtin_amdgcn_s_setprio(1);
    mm(0, 0);
    mm(0, 1);
    __builtin_amdgcn_s_setprio(0);
    if (!g1) wait_vm<8>();
    T4_BAR();
    loadA(cur, 1);  // phase B
    stage(sB[0], UB0, t + 2, b);
    stage(sB[1], UB1, t + 2, b);
    T4_LGKM0();
    if (g1) wait_vm<6>();
    T4_BAR();
    __builtin_amdgcn_s_setprio(1);
    mm(1, 1);
    mm(1, 0);
    __builtin_amdgcn_s_setprio(0);
    if (!g1) wait_vm<6>();
    T4_BAR();
  }
  if (!g1) T4_BAR();
#undef T4_BAR
#undef T4_LGKM0
  wait_vm<0>();  // never leave an LDS-DMA in flight past the end of the workgroup
  constexpr int OSZ = out_size<OUT>();
  const __amdgpu_buffer_rsrc_t crc =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.c, 0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t row = m0 + wr * 128 + (i >> 2) * 64 + (i & 3) * 16 + frow;
    char* crow = c_row<OSZ, CMODE == 2 ? 0 : 2>(p, row);
#pragma unroll
    for (int nq = 0; nq < 2; ++nq) {
      char* dst = crow + (n0 + wc * 64 + nq * 32 + fq * 8) * OSZ;
      // one store site (two branch-local stores get merged by the optimizer, which drops the
      // non-temporal hint)
      f32x4 v0 = acc[i][nq * 2], v1 = acc[i][nq * 2 + 1];
      if (p.act != ACT_NONE) {
        v0 = act4(v0, p.act);
        v1 = act4(v1, p.act);
      }
      if constexpr (CMODE == 2)
        store8_wt<OUT>(crc, (unsigned)(dst - (char*)p.c), v0, v1);
      else
        Store8<OUT>::st(dst, v0, v1);
    }
  }
}


// ---------------------------------------------------------------- pt4: persistent t4
// t4 streamed across a block's tiles (as pt8 does for t8). A tile's quadrants are stored right
// after their last MFMAs. Two schedules (see DEFER below):
//  * 16 / 8 reads (gated, CMODE 0 / 1): Q00 + Q01 after phase A of the tile's last K-tile,
//    Q11 + Q10 after phase B; vmcnt counts (NS = C store instructions per quadrant per wave):
//      normal:             A end 8,        B end 6
//      LAST of a tile:     A end g0 8+2NS / g1 8,   B end g0 6+4NS / g1 6+2NS
//      FIRST after a LAST: A end 8+4NS (both),      B end 6
//  * DEFER (12 / 12 reads): Q00 after phase A of the last K-tile, the other three after phase
//    B; every wait is 8, plus the stores issued after the unit it waits for (iter below).
// (stores count in issue order with the LDS-DMA; the counts keep exactly the ops issued after
// the unit the next phase reads in flight). Round 4 measured leaving the previous tile's stores
// in flight for one more phase of the next tile (KIND 2 waits 8 + 4 NS / 8 + 3 NS): neutral on
// every shape (profiles/r04/r4_7_ab_store_slack.txt): the store cost is CU-side issue, not the
// wait for the write acknowledgements.
// Load phases carry no VALU (round 3, profiles/r03/r3_20..r3_22: the un-prioritized loading wave
// pays ~90 cycles per VALU at the head of a segment, MI355X_MICROARCH.md "Two waves per SIMD"
// item 6; lab flagship 0.1093 -> 0.1039 ms, 8192^3 0.7555 -> 0.7286):
//  * LDS = [A units of buffers 0 / 1 | B units of buffers 0 / 1], unit (X, buf, q) at
//    X * 64K + buf * 32K + q * 16K: a fragment read is a fixed per-lane VGPR plus a compile-time
//    offset below 64 KB (the ds_read offset field); the buffer parity is static because every
//    tile has an even number of K-tiles and its body is unrolled by two (a run-time parity
//    branch between two instantiations made the register allocator spill ~250 VGPRs);
//  * LDS-DMA through buffer descriptors: per-tile panel base in SGPRs, K offset in soffset, the
//    per-lane source offsets fixed (pt4_ok keeps a 256-row panel below 2 GiB);
//  * CMODE 2 C stores through SGPR soffsets and one fixed per-lane voffset;
//  * a tile's first MFMA of every accumulator takes an inline-zero C operand (no v_mov zeroing).
// GATED: the arrival-flag form (a separate instantiation, so the ungated kernel's code and
// schedule are exactly those measured without flags).
// CMODE: 0 = grouped C rows, plain nt stores; 1 = C row-block table (direct store); 2 = grouped C
// rows in groups of a multiple of 256, write-through nt buffer stores (C's byte extent below
// 2 GiB: 32-bit offsets)
// APAN: A panels through grouped rows or a row-block table (a separate instantiation: deriving
// the panel base in the plain kernel cost it 6-16 more spilled SGPRs)
// KS: K-split (GemmArgs::ksplit slices, ungated, plain rows, CMODE 2): the virtual tiles are
// (slice, tile) pairs, slice-major; slice s reads A / B columns [s K, (s + 1) K) (K = the slice's
// length, lda / ldb the full rows) and stores its partial C at c + s * M * ldc (summed by the
// caller's reduce op): a few-tile long-K GEMM fills the chip in ONE launch
// (Retired in round 6, each measured slower than what stays, docs/RESULTS.md: the ONE schedule
// -- one section per K-tile and wave group, 0.6-2 % behind DEFER, r5_28 / r5_32; the K-split
// reduced inside the launch, ~10 % behind split + reduce op, r5_19; half-line C stores and the
// nt-only store policy, within noise, r5_22.)
template <class Mma, int OUT, bool GATED, int CMODE = 0, bool APAN = false, bool KS = false>
__global__ __launch_bounds__(512) void gemm_tn_pt4_kernel(const GemmArgs p) {
  constexpr int ROWB = 128, UNIT = 128 * ROWB;
  constexpr int NS = 4 * Store8<OUT>::kStores;
  constexpr int OSZ = out_size<OUT>();
  constexpr bool PAIR = is_pair<Mma>::value;
  // DEFER: the balanced schedule (ungated kernels): phase A reads the first halves (A rows mq = 0,
  // B cols nq = 0) and computes A0 x B0 plus the previous K-tile's A1 x B1, phase B the second
  // halves and A0 x B1 + A1 x B0; units are restaged as soon as both wave groups have read them
  // (6 intervals of DMA lead for every unit). Both halves' fragments stay live (+32 VGPRs: the
  // per-lane C addressing of CMODE 0 / 1 then spills). The gated kernels keep the 16 / 8-read
  // schedule too: they run the flagship shape, where the lab measured DEFER neutral
  // (profiles/r03/r3_27, r3_33), and their arrival gate sits at that schedule's A staging.
  constexpr bool DEFER = !GATED && CMODE == 2;
  constexpr int NH = DEFER ? 2 : 1;  // fragment register sets
  // tile_order 3 (own rows first, never gated) exists only for the RCCL-fed gated GEMM, whose A
  // is a row table (APAN): every other pt4 kernel compiles it out (SGPR pressure)
  constexpr bool OWN = GATED && APAN;
  // (DEFER 16-bit C: +32 KB, the parked C pairs, see PARK)
  __shared__ __attribute__((aligned(1024))) char smem[(DEFER && OUT != DT_F32 ? 10 : 8) * UNIT];
  // CMODE 2: C through one wave-uniform descriptor (launch_pt4 checks the extent fits)
  const __amdgpu_buffer_rsrc_t crc =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.c, 0, 0x7FFFFFF0, 0x00020000);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int nvt = KS ? ntiles * p.ksplit : ntiles;  // virtual tiles
  const int esz = Mma::kElem;
  const int nk = p.K * esz / ROWB;  // even (pt4_ok)
  int bid = (int)blockIdx.x, nblk = (int)gridDim.x;
  if constexpr (GATED && !APAN) {  // (the in-kernel all-gather reads plain A rows: gemm_launch)
    if (p.ag_ctas > 0) {  // in-kernel all-gather: the first ag_ctas workgroups copy
      if (bid < p.ag_ctas) {
        ag_copy_role<Mma::kElem>(p);
        return;
      }
      bid -= p.ag_ctas;
      nblk -= p.ag_ctas;
    }
  }
  const int my_tiles = (bid < nvt) ? (nvt - 1 - bid) / nblk + 1 : 0;
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
      offA[q][i] = (unsigned)(lr * p.lda * esz + ch);
      const int lc = (ur >> 5) * 64 + q * 32 + t8_perm(ur & 31);
      offB[q][i] = (unsigned)(lc * p.ldb * esz + ch);
    }
  }
  __amdgpu_buffer_rsrc_t rsA = crc, rsB = crc;  // set at the first stage
  int src_tile = -1;
  // A panel of a tile (its 256 logical rows are contiguous physical rows, pt4_ok): APAN = grouped
  // rows (groups of a multiple of 256 rows) or a row-block address table (blocks of a multiple of
  // 256 rows, e.g. the peers' IPC-mapped shards or a stage-major gather buffer); wave-uniform,
  // once per tile, with the tile's origin. The arrival gate indexes PHYSICAL rows of grouped A and
  // LOGICAL rows of a table.
  auto a_panel = [&](int64_t m0) __attribute__((always_inline)) -> const char* {
    if (APAN && p.a_table != nullptr) {
      const unsigned ur = (unsigned)m0, us = (unsigned)p.shard_rows, sh = ur / us;
      return (const char*)p.a_table[sh] + (int64_t)(ur - sh * us) * p.lda * esz;
    }
    return (const char*)p.a + (APAN ? map_row(m0, p.a_grp, p.a_gstride) : m0) * p.lda * esz;
  };
  auto flag_row = [&](int64_t m0) __attribute__((always_inline)) -> int64_t {
    if constexpr (!APAN) return m0;
    return p.a_table != nullptr ? m0 : map_row(m0, p.a_grp, p.a_gstride);
  };
  const char* na = nullptr;  // APAN: the next tile's A panel
  int64_t nko = 0;           // KS: the next tile's K-slice byte offset into the A / B rows
  unsigned ncs = 0, ccs = 0;  // KS: the next / current tile's partial-C byte offset
  auto origin = [&](int ti, int64_t& m0, int64_t& n0) __attribute__((always_inline)) {
    int wg = tile_index_virtual<OWN>(p, bid + ti * nblk, nvt);
    if constexpr (KS) {
      const int ks = wg / ntiles;
      wg -= ks * ntiles;
      nko = (int64_t)ks * p.K * esz;
      ncs = (unsigned)((int64_t)ks * p.M * p.ldc * OSZ);
    }
    int tm_, tn_;
    tile_mn(p, wg, p.M / 256, tiles_n, tm_, tn_);
    m0 = (int64_t)tm_ * 256;
    n0 = (int64_t)tn_ * 256;
    if constexpr (APAN) na = a_panel(m0);
  };
  // Tile origins are computed once per tile, at its start, for the tile itself (stores) and for
  // the next one (staging runs up to two K-tiles ahead, arrival gate): the index maps' integer
  // divisions would otherwise be inlined at every stage / store site (code size, I-cache).
  int64_t cm0 = 0, cn0 = 0, nm0 = 0, nn0 = 0;
  origin(0, nm0, nn0);
  struct Cur { int ti, kt; };
  auto adv = [&](Cur& c) __attribute__((always_inline)) {
    if (c.ti == my_tiles - 1 && c.kt == nk - 1) return;
    if (++c.kt == nk) { c.kt = 0; ++c.ti; }
  };
  // LDS unit (X = 0 A / 1 B, buffer, half q)
  auto uoff = [](int X, int buf, int q) constexpr { return X * 65536 + buf * 32768 + q * 16384; };
  auto stage_dma = [&](int X, int q, int buf, Cur c) __attribute__((always_inline)) {
    const unsigned* off = X == 0 ? offA[q] : offB[q];
    char* dst = smem + uoff(X, buf, q) + wave * 16 * ROWB;
    const unsigned soff = (unsigned)(c.kt * ROWB);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(X == 0 ? rsA : rsB, (LDS_AS void*)dst, 16, off[0],
                                             soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(X == 0 ? rsA : rsB, (LDS_AS void*)(dst + 8 * ROWB),
                                             16, off[1], soff, 0, 0);
  };
  auto stage = [&](int X, int q, int buf, Cur c) __attribute__((always_inline)) {
    if (c.ti != src_tile) {  // always the next tile (nm0, nn0)
      rsA = __builtin_amdgcn_make_buffer_rsrc((void*)((APAN ? na : a_panel(nm0)) + (KS ? nko : 0)),
                                              0, 0x7FFFFFF0, 0x00020000);
      rsB = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((const char*)p.b + nn0 * p.ldb * esz + (KS ? nko : 0)), 0, 0x7FFFFFF0,
          0x00020000);
      src_tile = c.ti;
    }
    stage_dma(X, q, buf, c);
  };
  // Both units (A, B) of half q of K-tile c. SAME: c is a K-tile of the tile whose descriptors
  // are current (the steady loop's iterations but its last), so the tile-change test -- 8
  // s_cselect per load phase -- is compiled out: bf16 -0.8 to -2.3 % on the flagship, K = 4096,
  // K = 512 and 8192^3, MX flat (profiles/r06/r6_28, r6_29)
  auto stage_ab = [&](auto same_tag, int q, int buf, Cur c) __attribute__((always_inline)) {
    if constexpr (decltype(same_tag)::value) {
      stage_dma(0, q, buf, c);
      stage_dma(1, q, buf, c);
    } else {
      stage(0, q, buf, c);
      stage(1, q, buf, c);
    }
  };
  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;
  const int c0 = ((0 + fq) ^ sw) * 16, c1 = ((4 + fq) ^ sw) * 16;
  unsigned rA0 = (wr * 64 + frow) * ROWB + c0, rA1 = (wr * 64 + frow) * ROWB + c1;
  constexpr unsigned BBASE = 65536;  // start of the B units
  unsigned rB0 = BBASE + (wc * 32 + frow) * ROWB + c0, rB1 = BBASE + (wc * 32 + frow) * ROWB + c1;
  // opaque bases: otherwise the B base's 64K can be re-associated into a read's constant, which
  // then no longer fits the ds_read offset field (a VGPR per read)
  asm volatile("" : "+v"(rA0), "+v"(rA1), "+v"(rB0), "+v"(rB1));
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x4 aR[NH][4][2], bR[2][2][2];  // [A half (DEFER) / 0][frag][k16], [B half][frag][k16]
  i32x8 aP[NH][4], bP[2][2];
  auto loadA = [&](auto bufc, int mq) __attribute__((always_inline)) {
    constexpr int BUF = decltype(bufc)::value;
    const int h = DEFER ? mq : 0;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int o = uoff(0, BUF, mq) + f * 16 * ROWB;
      if constexpr (PAIR) {
        aP[h][f].lo = *(const i32x4*)(smem + rA0 + o);
        aP[h][f].hi = *(const i32x4*)(smem + rA1 + o);
      } else {
        aR[h][f][0] = *(const i32x4*)(smem + rA0 + o);
        aR[h][f][1] = *(const i32x4*)(smem + rA1 + o);
      }
    }
  };
  auto loadB = [&](auto bufc, int nq) __attribute__((always_inline)) {
    constexpr int BUF = decltype(bufc)::value;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int o = uoff(0, BUF, nq) + g * 16 * ROWB;  // rB0 / rB1 carry the B region's 64K
      if constexpr (PAIR) {
        bP[nq][g].lo = *(const i32x4*)(smem + rB0 + o);
        bP[nq][g].hi = *(const i32x4*)(smem + rB1 + o);
      } else {
        bR[nq][g][0] = *(const i32x4*)(smem + rB0 + o);
        bR[nq][g][1] = *(const i32x4*)(smem + rB1 + o);
      }
    }
  };
  // zero: the tile's first K-tile; each accumulator's first MFMA takes an inline-zero C operand
  auto mm = [&](int mq, int nq, bool zero) __attribute__((always_inline)) {
    const int h = DEFER ? mq : 0;
    if constexpr (PAIR) {
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          if (zero) acc[mq * 4 + f][nq * 2 + g] = f32x4{0.f, 0.f, 0.f, 0.f};
          Mma::step8(acc[mq * 4 + f][nq * 2 + g], bP[nq][g], aP[h][f]);
        }
#pragma unroll
      for (int f = 0; f < 4; ++f)  // pin the pure scaled MFMAs in this section (see t8)
#pragma unroll
        for (int g = 0; g < 2; ++g) asm volatile("" : "+v"(acc[mq * 4 + f][nq * 2 + g]));
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
          for (int g = 0; g < 2; ++g) {
            if (zero && kk == 0) acc[mq * 4 + f][nq * 2 + g] = f32x4{0.f, 0.f, 0.f, 0.f};
            Mma::step(acc[mq * 4 + f][nq * 2 + g], bR[nq][g][kk], aR[h][f][kk]);
          }
    }
  };
  int ti = 0;
  // CMODE 2: the lane's part of a C offset (fixed) and the wave-uniform part per fragment row
  const unsigned c_lane = (unsigned)(((wr * 128 + frow) * p.ldc + wc * 64 + fq * 8) * OSZ);
  // (no fused activation: pt4_ok routes those GEMMs to t4, keeping pt4's code small)
  auto store_q = [&](int mq, int nq) __attribute__((always_inline)) {
    const int64_t m0 = cm0, n0 = cn0;
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int i = mq * 4 + f;
      const f32x4 v0 = acc[i][nq * 2], v1 = acc[i][nq * 2 + 1];
      if constexpr (CMODE == 2) {
        // grouped C rows: a tile's 256 rows stay contiguous (launch_pt4: c_grp % 256 == 0)
        const int64_t prow = m0 + mq * 64 + f * 16;  // cm0: already the physical row
        const unsigned soff = (unsigned)((prow * p.ldc + n0 + nq * 32) * OSZ) + (KS ? ccs : 0u);
        store8_wt<OUT>(crc, c_lane, v0, v1, soff);
      } else {
        const int64_t row = m0 + wr * 128 + mq * 64 + f * 16 + frow;
        char* dst = c_row<OSZ, CMODE == 1 ? 1 : 0>(p, row) +
                    (n0 + wc * 64 + nq * 32 + fq * 8) * OSZ;
        Store8<OUT>::st(dst, v0, v1);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  // PAIRST (DEFER, 16-bit C): a tile's C leaves in whole 128-byte lines. A lane holds 16 B of row
  // frow in each 32-column quadrant (nq 0 / 1: bytes 16 fq and 64 + 16 fq of the wave's 128-byte
  // row slice); one DPP row_ror:8 per dword, masked to half the lanes, gives lanes 8-15 of every
  // 16-lane row the quadrant-1 chunk of row frow - 8 (X) and lanes 0-7 the quadrant-0 chunk of
  // row frow + 8 (Y), so X covers rows 0-7 and Y rows 8-15 of the fragment, 128 contiguous bytes
  // per row each (lab: a 128 MB write-through stream 23.1-24.5 us vs 25.1-25.8 us in half lines,
  // nt only 20.8-22.0 vs 38.1-40.1 us, profiles/r05/r5_21_store_pattern.txt).
  constexpr bool PAIRST = DEFER && OUT != DT_F32;
  // Cache policy of those stores: sc1 | nt (write-through, no L2 allocation), except for the
  // block-scaled MX-fp8 kernel, whose tiles end twice as often (8 K-tiles per 1024-deep tile):
  // sc0 | sc1 there, 2.3 % and 3.5 % faster on the MX flagship in two sessions (and 5-6 %
  // slower for bf16, which keeps sc1 | nt; profiles/r06/r6_3_*, r6_4_*; lab variants auxN)
  constexpr int CPOL = std::is_same<Mma, MmaMX>::value ? 17 : 18;
  const unsigned c_pair =
      (unsigned)(((wr * 128 + (frow & 7)) * p.ldc + wc * 64) * OSZ + ((frow & 8) ? 64 : 0) +
                 fq * 16);
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
  // PARK (PAIRST): a tile's last NP of its 4 NS C stores per wave (rows mq = 1, f = 2, 3) go to
  // LDS beside the staging buffers (4 KB per wave, the wave's own) and leave in the next tile's
  // first K-tile, 2 after each load phase's DMA. The store path drains only ~12.6 B/clk per CU
  // whatever the rest of the chip does (32 or 256 CUs storing alike, profiles/r06/r6_8), and the
  // vmcnt of the next DMA waits count the stores issued before it: the tile-end interval is a
  // queue of C stores, a quarter of which now leaves beside the next tile's MFMAs.
  // (A workgroup's last tile drains its parked pairs at the end.)
  constexpr bool PARK = PAIRST;
  constexpr int NP = PARK ? 4 : 0;
  constexpr int PBASE = 8 * UNIT;
  unsigned pso = 0;  // the parked tile's C offset (its row 0, column 0, K-split partial)
  auto park_read = [&](int j0, u32x4_t (&v)[2]) __attribute__((always_inline)) {
    v[0] = *(const u32x4_t*)(smem + PBASE + wave * 4096 + j0 * 1024 + lane * 16);
    v[1] = *(const u32x4_t*)(smem + PBASE + wave * 4096 + (j0 + 1) * 1024 + lane * 16);
  };
  auto park_store = [&](int j0, const u32x4_t (&v)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int jx = j0 + jj, f = 2 + (jx >> 1);  // slot: x (even) / y (odd, rows + 8) of f
      const unsigned so = pso + (unsigned)((64 + f * 16 + ((jx & 1) ? 8 : 0)) * p.ldc * OSZ);
      __builtin_amdgcn_raw_buffer_store_b128(v[jj], crc, c_pair, so, CPOL);
    }
  };
  auto store_pair = [&](int mq) __attribute__((always_inline)) {
    if constexpr (PAIRST) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const int i = mq * 4 + f;
        u32x4_t x = pack8<OUT>(acc[i][0], acc[i][1]), y = pack8<OUT>(acc[i][2], acc[i][3]);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int t = (int)x[d];
          x[d] = (unsigned)__builtin_amdgcn_update_dpp(t, (int)y[d], 0x128, 0xF, 0xC, false);
          y[d] = (unsigned)__builtin_amdgcn_update_dpp((int)y[d], t, 0x128, 0xF, 0x3, false);
        }
        if (PARK && mq == 1 && f >= 2) {
          char* pp = smem + PBASE + wave * 4096 + (f - 2) * 2048 + lane * 16;
          *(u32x4_t*)pp = x;
          *(u32x4_t*)(pp + 1024) = y;
        } else {
          const int64_t prow = cm0 + mq * 64 + f * 16;
          const unsigned so = (unsigned)((prow * p.ldc + cn0) * OSZ) + (KS ? ccs : 0u);
          const unsigned so8 = so + (unsigned)(8 * p.ldc * OSZ);
          __builtin_amdgcn_raw_buffer_store_b128(x, crc, c_pair, so, CPOL);
          __builtin_amdgcn_raw_buffer_store_b128(y, crc, c_pair, so8, CPOL);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
#define T4_BAR()                         \
  do {                                   \
    __builtin_amdgcn_sched_barrier(0);   \
    __builtin_amdgcn_s_barrier();        \
    __builtin_amdgcn_sched_barrier(0);   \
  } while (0)
// lgkmcnt(0) through the builtin (vmcnt / expcnt at their maxima, pinned by scheduling
// barriers): the compiler's waitcnt pass sees it, so it does not re-wait, counted, for reads it
// believes still in flight at the head of the next MFMA phase
#define T4_LGKM0()                            \
  do {                                        \
    __builtin_amdgcn_sched_barrier(0);        \
    __builtin_amdgcn_s_waitcnt(0xC07F);       \
    __builtin_amdgcn_sched_barrier(0);        \
  } while (0)
  const bool g1 = wr == 1;  // wave-uniform (wave came through readfirstlane)
  if constexpr (GATED) {  // arrival gate of the first tile
    const int64_t f0 = flag_row(nm0);
    wait_flag<OWN>(p, f0, f0 + 255);
  }
  Cur q0{0, 0}, q1{0, 0};
  adv(q1);
  if constexpr (DEFER) {
    stage(0, 0, 0, q0);  // halves 0 of K-tile 0 ("phase B of K-tile -2")
    stage(1, 0, 0, q0);
    stage(0, 1, 0, q0);  // halves 1 of K-tile 0 ("phase A of K-tile -1")
    stage(1, 1, 0, q0);
    stage(0, 0, 1, q1);  // halves 0 of K-tile 1 ("phase B of K-tile -1")
    stage(1, 0, 1, q1);
  } else {
    stage(1, 0, 0, q0);
    stage(1, 1, 0, q0);
    stage(0, 0, 0, q0);
    stage(0, 1, 0, q0);
    stage(1, 0, 1, q1);
    stage(1, 1, 1, q1);
  }
  // DEFER: qa = K-tile t+1 (halves 1, phase A), qb = t+2 (halves 0, phase B); otherwise qa = t+1
  // (A units, phase A), qb = t+2 (B units, phase B)
  Cur qa = q1, qb = q1;
  adv(qb);
  wait_vm<DEFER ? 8 : 6>();
  T4_BAR();
  if (g1) T4_BAR();
  // KIND: 0 normal, 1 last K-tile of a tile, 2 first K-tile after a tile's last, 4 the kernel's
  // first K-tile (DEFER: no deferred product, no stores counted); BUF: the buffer this K-tile
  // reads. vmcnt counts keep exactly the DMA (and C stores) issued after the units the next phase
  // reads in flight; stores count in issue order with the DMA.
  // SAME (same_tag): qa and qb stay inside the current tile (stage_ab, cursor advance); G1: this
  // wave's group, a compile-time tag where the tile loop is split per group (SPLIT, below)
  auto iter = [&](auto bufc, auto kind_tag, auto same_tag, auto g1v) __attribute__((always_inline)) {
    constexpr int KIND = decltype(kind_tag)::value;
    constexpr bool SAME = decltype(same_tag)::value;
    const bool g1 = g1v;
    constexpr int BUF = decltype(bufc)::value;
    constexpr bool Z = KIND == 2 || KIND == 4;
    if constexpr (DEFER) {
      constexpr bool DEF = KIND == 0 || KIND == 1;  // previous K-tile's A1 x B1
      // MFMA phases at raised wave priority for the MX kernel only: without it the 16-bit
      // kernels ran 0.2-1.1 % faster on all 8 shapes of two sessions (flagship, K = 4096 / 8192,
      // 8192^3, 16384x8192x8192), MX-fp8 flat to 0.9 % slower (profiles/r06/r6_18, r6_19)
      constexpr bool PRIO = std::is_same<Mma, MmaMX>::value;
      // PARK waits: the previous tile's 4 NS - NP direct stores, then per load phase 4 DMA + 2
      // parked stores
      constexpr int WK2A = PARK ? 8 + 4 * NS - NP + 2 : 8 + 3 * NS;
      constexpr int WK2B = PARK ? 8 + 4 * NS - NP + 4 : 8;
      u32x4_t pv[2];
      loadB(bufc, 0);  // phase A: halves 0
      loadA(bufc, 0);
      if constexpr (PARK && KIND == 2) park_read(0, pv);
      stage_ab(same_tag, 1, BUF ^ 1, qa);
      T4_LGKM0();
      if constexpr (PARK && KIND == 2) park_store(0, pv);
      if (g1) wait_vm<KIND == 2 ? WK2A : 8>();
      T4_BAR();
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
      if constexpr (DEF) mm(1, 1, false);
      mm(0, 0, Z);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      // (PAIRST: every store after phase B, the first pair needs quadrant (0, 1); the counts of
      // the two waits below then drop the NS stores issued here before)
      if constexpr (KIND == 1 && !PAIRST) store_q(0, 0);
      if (!g1) wait_vm<KIND == 2 ? WK2A : (KIND == 1 && !PAIRST ? 8 + NS : 8)>();
      T4_BAR();
      loadB(bufc, 1);  // phase B: halves 1
      loadA(bufc, 1);
      if constexpr (PARK && KIND == 2) park_read(2, pv);
      stage_ab(same_tag, 0, BUF, qb);
      T4_LGKM0();
      if constexpr (PARK && KIND == 2) park_store(2, pv);
      if (g1) wait_vm<KIND == 2 ? WK2B : (KIND == 1 && !PAIRST ? 8 + NS : 8)>();
      T4_BAR();
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
      mm(0, 1, Z);
      // PAIRST: rows mq = 0 are final here; storing them now frees their accumulators before
      // the rest of the phase (held to the end of the phase they spilled 52 bytes)
      if constexpr (KIND == 1 && PAIRST) store_pair(0);
      mm(1, 0, Z);
      if constexpr (KIND == 1) mm(1, 1, false);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      if constexpr (KIND == 1 && PAIRST) {
        if constexpr (PARK) pso = (unsigned)((cm0 * p.ldc + cn0) * OSZ) + (KS ? ccs : 0u);
        store_pair(1);  // 4 NS stores in all (NP of them parked), as the quadrant form's
      } else if constexpr (KIND == 1) {
        store_q(0, 1);
        store_q(1, 0);
        store_q(1, 1);
      }
      if constexpr (KIND == 1) {
#pragma unroll
        for (int f = 0; f < 4; ++f) {  // the next tile's first A1 x B1 is a deferred product
          acc[4 + f][2] = f32x4{0.f, 0.f, 0.f, 0.f};
          acc[4 + f][3] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      if (!g1) wait_vm<KIND == 1 ? 8 + 4 * NS - NP : (KIND == 2 ? WK2B : 8)>();
      T4_BAR();
    } else {
      if (GATED && qa.kt == 0) {
        // Arrival gate: this iteration stages the first A K-tile of tile qa.ti. Thread 0 spins on
        // the flags of its rows and acquires; one extra barrier, executed by every wave at this
        // same point (qa is workgroup-uniform), orders all waves' A staging after it. Both wave
        // groups insert it at the same place, so their one-barrier stagger is unchanged; an extra
        // barrier only adds ordering (LDS RAW / WAR distances grow).
        const int64_t f0 = flag_row(nm0);  // qa.ti is the next tile (or tile 0)
        wait_flag_t0<OWN>(p, f0, f0 + 255);
        T4_BAR();
      }
      loadB(bufc, 0);  // phase A
      loadB(bufc, 1);
      loadA(bufc, 0);
      stage(0, 0, BUF ^ 1, qa);
      stage(0, 1, BUF ^ 1, qa);
      T4_LGKM0();
      if (g1) wait_vm<KIND == 2 ? 8 + 4 * NS : 8>();
      T4_BAR();
      __builtin_amdgcn_s_setprio(1);
      mm(0, 0, Z);
      mm(0, 1, Z);
      __builtin_amdgcn_s_setprio(0);
      if constexpr (KIND == 1) {
        store_q(0, 0);
        store_q(0, 1);
      }
      if (!g1) wait_vm<KIND == 1 ? 8 + 2 * NS : (KIND == 2 ? 8 + 4 * NS : 8)>();
      T4_BAR();
      loadA(bufc, 1);  // phase B
      stage(1, 0, BUF, qb);
      stage(1, 1, BUF, qb);
      T4_LGKM0();
      if (g1) wait_vm<KIND == 1 ? 6 + 2 * NS : 6>();
      T4_BAR();
      __builtin_amdgcn_s_setprio(1);
      mm(1, 1, Z);
      mm(1, 0, Z);
      __builtin_amdgcn_s_setprio(0);
      if constexpr (KIND == 1) {
        store_q(1, 1);
        store_q(1, 0);
      }
      if (!g1) wait_vm<KIND == 1 ? 6 + 4 * NS : 6>();
      T4_BAR();
    }
    qa = qb;
    if constexpr (SAME)
      ++qb.kt;
    else
      adv(qb);
  };
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;
  auto tile_body = [&](auto first_kind, auto last_kind, auto g1v) __attribute__((always_inline)) {
    cm0 = nm0;  // this tile (C rows: physical, grouped C rows keep a tile contiguous)
    cn0 = nn0;
    if constexpr (KS) ccs = ncs;
    if constexpr (CMODE == 2) cm0 = map_row(cm0, p.c_grp, p.c_gstride);
    if (ti + 1 < my_tiles) origin(ti + 1, nm0, nn0);
    using InTile = std::true_type;
    using Crosses = std::false_type;
    iter(B0{}, first_kind, Crosses{}, g1v);  // K-tile 0
    int t = 1;
    for (; t + 4 < nk; t += 2) {  // qb <= K-tile t + 3 <= nk - 2: this tile
      iter(B1{}, K0{}, InTile{}, g1v);
      iter(B0{}, K0{}, InTile{}, g1v);
    }
    if (t + 2 < nk) {  // the last pair stages the next tile's first K-tile
      iter(B1{}, K0{}, Crosses{}, g1v);
      iter(B0{}, K0{}, Crosses{}, g1v);
    }
    iter(B1{}, last_kind, Crosses{}, g1v);  // K-tile nk - 1 (nk even)
  };
  auto tiles = [&](auto g1v) __attribute__((always_inline)) {
    ti = 0;
    tile_body(std::integral_constant<int, DEFER ? 4 : 0>{}, K1{}, g1v);
    for (ti = 1; ti < my_tiles; ++ti) tile_body(std::integral_constant<int, 2>{}, K1{}, g1v);
  };
  // SPLIT: the tile loop instantiated once per wave group, so every `if (g1)` around a vmcnt
  // wait folds away (no branch per phase): bf16 flagship -1.9 %, 8192^3 -1.7 %, K = 512 -4.1 %
  // (profiles/r06/r6_30, r6_31). The MX, row-table (APAN), f32-output and gated forms spill
  // with two copies of the loop (MX 72-76 bytes and 37-67 % slower, f32 C 8 bytes) and keep one
  constexpr bool SPLIT = DEFER && !APAN && OUT != DT_F32 && !std::is_same<Mma, MmaMX>::value;
  if constexpr (SPLIT) {
    if (g1)
      tiles(std::true_type{});
    else
      tiles(std::false_type{});
  } else {
    tiles(g1);
  }
  if (!g1) T4_BAR();
  if constexpr (PARK) {  // the last tile's parked pairs
    u32x4_t pv[2];
    park_read(0, pv);
    park_store(0, pv);
    park_read(2, pv);
    park_store(2, pv);
  }
#undef T4_BAR
#undef T4_LGKM0
  wait_vm<0>();  // never leave an LDS-DMA in flight past the end of the workgroup
}

// ---------------------------------------------------------------- pt8: persistent t8
// One workgroup per CU streams its tiles' K-tiles back to back (stream index h = tile * nk + kt;
// the t8 unit schedule above runs unchanged across tile boundaries, so only the first tile pays
// the staging fill). A tile's C quadrants are stored right after their last MFMAs (quadrant (0,0)
// in phase 0 of the tile's last K-tile, ..., (1,0) in phase 3), which spreads the C burst over a
// K-tile; the stores issued after that K-tile's UB0 stage are allowed to stay in flight across
// its vmcnt (vmcnt counts loads, LDS-DMA and stores together, in issue order). The stage cursors
// advance incrementally (no integer division in the loop) and the tile's last K-tile is a
// separate instantiation of the body, so the steady-state loop carries no store code.
// Measured (research/lab, profiles/r01/s2/lab/): 65536x1024x1024 bf16 0.1116 ms vs t8 0.1163.
template <class Mma, int OUT>
__global__ __launch_bounds__(512) void gemm_tn_pt8_kernel(const GemmArgs p) {
  constexpr int ROWB = 128, UNIT = 128 * ROWB, STAGE = 4 * UNIT;
  constexpr int UA0 = 0, UA1 = UNIT, UB0 = 2 * UNIT, UB1 = 3 * UNIT;
  constexpr int NS = 4 * Store8<OUT>::kStores;  // C store instructions per quadrant per wave
  constexpr int OSZ = out_size<OUT>();
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int tiles_n = p.N / 256, ntiles = (p.M / 256) * tiles_n;
  const int esz = Mma::kElem;
  const int nk = p.K * esz / ROWB;
  const int my_tiles =
      ((int)blockIdx.x < ntiles) ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  if (my_tiles == 0) return;

  const int drow = lane >> 3, dpc = lane & 7;
  const char* sA[2][2];
  const char* sB[2][2];
  int src_tile = -1;
  auto tile_origin = [&](int ti, int64_t& m0, int64_t& n0) __attribute__((always_inline)) {
    const int wg = tile_index_virtual(p, (int)blockIdx.x + ti * (int)gridDim.x, ntiles);
    int tm_, tn_;
    tile_mn(p, wg, p.M / 256, tiles_n, tm_, tn_);
    m0 = (int64_t)tm_ * 256;
    n0 = (int64_t)tn_ * 256;
  };
  auto set_src = [&](int ti) __attribute__((always_inline)) {
    int64_t m0, n0;
    tile_origin(ti, m0, n0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ur = wave * 16 + i * 8 + drow;
      const int ch = (dpc ^ ((ur >> 1) & 7)) * 16;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int lr = (ur >> 6) * 128 + q * 64 + (ur & 63);
        sA[q][i] = a_row(p, m0 + lr, esz) + ch;
        const int lc = (ur >> 5) * 64 + q * 32 + t8_perm(ur & 31);
        sB[q][i] = (const char*)p.b + (n0 + lc) * p.ldb * esz + ch;
      }
    }
  };
  // stage stream cursors: (tile, K-tile) of h+1 and h+2, clamped to the last K-tile of the last
  // tile past the end of the stream (identical bytes into units no one reads again)
  struct Cur { int ti, kt; };
  auto adv = [&](Cur& c) __attribute__((always_inline)) {
    if (c.ti == my_tiles - 1 && c.kt == nk - 1) return;
    if (++c.kt == nk) { c.kt = 0; ++c.ti; }
  };
  auto stage = [&](int which, int unit_off, Cur c, int buf) __attribute__((always_inline)) {  // 0/1: A mq0/mq1, 2/3: B nq0/nq1
    if (c.ti != src_tile) {
      set_src(c.ti);
      src_tile = c.ti;
    }
    const char* const* src = which < 2 ? sA[which] : sB[which - 2];
    char* dst = smem + buf * STAGE + unit_off + wave * 16 * ROWB;
    glds16(src[0] + (int64_t)c.kt * ROWB, dst);
    glds16(src[1] + (int64_t)c.kt * ROWB, dst + 8 * ROWB);
  };

  const int frow = lane & 15, fq = lane >> 4, sw = (frow >> 1) & 7;
  const int c0 = ((0 + fq) ^ sw) * 16, c1 = ((4 + fq) ^ sw) * 16;
  const int aoff = (wr * 64 + frow) * ROWB, boff = (wc * 32 + frow) * ROWB;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x4 aR[4][2], bR[2][2];  // fragments: [f or g][K-half]
  i32x8 aP[4], bP[2];        // MX (kPair): both K-halves in one register tuple, loaded in place
  constexpr bool PAIR = is_pair<Mma>::value;
  auto loadA = [&](const char* base, int mq) __attribute__((always_inline)) {
    const char* r = base + (mq ? UA1 : UA0) + aoff;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      if constexpr (PAIR) {
        aP[f].lo = *(const i32x4*)(r + f * 16 * ROWB + c0);
        aP[f].hi = *(const i32x4*)(r + f * 16 * ROWB + c1);
      } else {
        aR[f][0] = *(const i32x4*)(r + f * 16 * ROWB + c0);
        aR[f][1] = *(const i32x4*)(r + f * 16 * ROWB + c1);
      }
    }
  };
  auto loadB = [&](const char* base, int nq) __attribute__((always_inline)) {
    const char* r = base + (nq ? UB1 : UB0) + boff;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if constexpr (PAIR) {
        bP[g].lo = *(const i32x4*)(r + g * 16 * ROWB + c0);
        bP[g].hi = *(const i32x4*)(r + g * 16 * ROWB + c1);
      } else {
        bR[g][0] = *(const i32x4*)(r + g * 16 * ROWB + c0);
        bR[g][1] = *(const i32x4*)(r + g * 16 * ROWB + c1);
      }
    }
  };
  auto comp = [&](int mq, int nq) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    if constexpr (PAIR) {  // one MFMA per 128-byte K-row
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g) Mma::step8(acc[mq * 4 + f][nq * 2 + g], bP[g], aP[f]);
      // The scaled MFMA is a pure intrinsic: without a use here LLVM sinks all four phases' MFMAs
      // past the barriers to the end of the K-tile (observed: 32 back-to-back MFMAs, spills and
      // vmcnt(0) drains in the loop). An empty asm that "modifies" the quadrant's accumulators
      // pins them inside this phase's compute section.
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 2; ++g) asm volatile("" : "+v"(acc[mq * 4 + f][nq * 2 + g]));
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
          for (int g = 0; g < 2; ++g) Mma::step(acc[mq * 4 + f][nq * 2 + g], bR[g][kk], aR[f][kk]);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  int ti = 0;
  auto store_q = [&](int mq, int nq) __attribute__((always_inline)) {  // store + clear quadrant (mq, nq) of tile ti
    int64_t m0, n0;
    tile_origin(ti, m0, n0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int i = mq * 4 + f;
      const int64_t row = m0 + wr * 128 + mq * 64 + f * 16 + frow;
      char* dst = c_row<OSZ>(p, row) +
                  (n0 + wc * 64 + nq * 32 + fq * 8) * OSZ;
      // one store site (two branch-local stores get merged by the optimizer, which drops the
      // non-temporal hint)
      f32x4 v0 = acc[i][nq * 2], v1 = acc[i][nq * 2 + 1];
      if (p.act != ACT_NONE) {
        v0 = act4(v0, p.act);
        v1 = act4(v1, p.act);
      }
      Store8<OUT>::st(dst, v0, v1);
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
  adv(q1);
  stage(0, UA0, q0, 0);
  stage(3, UB1, q0, 0);
  stage(1, UA1, q0, 0);
  stage(2, UB0, q0, 0);
  stage(0, UA0, q1, 1);
  stage(3, UB1, q1, 1);
  Cur q2 = q1;
  adv(q2);
  wait_vm<4>();
  T8_BAR();
  const bool g1 = wr == 1;  // wave-uniform (wave came through readfirstlane)
  if (g1) T8_BAR();
  // one K-tile of the stream; LAST = the tile's last K-tile (stores its quadrants)
  auto iter = [&](int h, auto last_tag) __attribute__((always_inline)) {
    constexpr bool LAST = decltype(last_tag)::value;
    const int b = h & 1, nb = b ^ 1;
    const char* cur = smem + b * STAGE;
    loadA(cur, 0);  // p0
    loadB(cur, 0);
    stage(1, UA1, q1, nb);
    T8_BAR();
    comp(0, 0);
    if constexpr (LAST) store_q(0, 0);
    T8_BAR();
    loadB(cur, 1);  // p1
    stage(2, UB0, q1, nb);
    T8_BAR();
    comp(0, 1);
    if constexpr (LAST) store_q(0, 1);
    T8_BAR();
    loadA(cur, 1);  // p2
    stage(0, UA0, q2, b);
    T8_BAR();
    comp(1, 1);
    if constexpr (LAST) store_q(1, 1);
    T8_BAR();
    loadB(cur, 0);  // p3
    stage(3, UB1, q2, b);
    // younger than UB0(h+1): UA0/UB1(h+2) and, in a tile's last K-tile, the Q01 + Q11 stores
    if (g1) wait_vm<LAST ? 4 + 2 * NS : 4>();
    T8_BAR();
    comp(1, 0);
    if constexpr (LAST) store_q(1, 0);
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
  wait_vm<0>();  // never leave an LDS-DMA in flight past the end of the workgroup
}

// ---------------------------------------------------------------- MX-fp8 (block-scaled) kernel
// One v_mfma_scale_f32_16x16x128_f8f6f4 per 128-byte K-row (unit E8M0 scales = 127): 2x the bf16
// MFMA rate (MI355X_MICROARCH.md "Matrix cores"). Same staging as above.
template <int OUT, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM* WN * 64) void gemm_tn_mxfp8_kernel(const GemmArgs p) {
  constexpr int NW = WM * WN, ROWB = 128;
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE = A_BYTES + B_BYTES;
  constexpr int TM = BM / WM, TN = BN / WN, MR = TM / 16, NR = TN / 16;
  constexpr int LA = BM / 8 / NW, LB = BN / 8 / NW;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int wg = tile_index(p, nwg);
  const int tm = wg / tiles_n, tn = wg % tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const char* aptr[LA];
  const char* bptr[LB];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    const int row = (wave * LA + i) * 8 + (lane >> 3);
    int64_t gr = m0 + row;
    gr = gr < p.M ? gr : p.M - 1;
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    aptr[i] = (const char*)p.a + map_row(gr, p.a_grp, p.a_gstride) * p.lda + chunk * 16;
  }
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int row = (wave * LB + i) * 8 + (lane >> 3);
    int64_t gr = n0 + row;
    gr = gr < p.N ? gr : p.N - 1;
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    bptr[i] = (const char*)p.b + gr * p.ldb + chunk * 16;
  }
  wait_tile(p, m0, BM);
  auto stage = [&](int buf, int kt) __attribute__((always_inline)) {
    char* base = smem + buf * STAGE;
    const int64_t koff = (int64_t)kt * ROWB;
#pragma unroll
    for (int i = 0; i < LA; ++i) glds16(aptr[i] + koff, base + (wave * LA + i) * 1024);
#pragma unroll
    for (int i = 0; i < LB; ++i) glds16(bptr[i] + koff, base + A_BYTES + (wave * LB + i) * 1024);
  };
  const int wm = wave / WN, wn = wave % WN;
  const int swz = (lane & 15) >> 1, frow = lane & 15, fq = lane >> 4;
  f32x4 acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES;
    const int c0 = ((fq) ^ swz) * 16, c1 = ((4 + fq) ^ swz) * 16;
    i32x8 af[MR], bfr[NR];
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const char* r = As + (wm * TM + i * 16 + frow) * ROWB;
      const i32x4 lo = *(const i32x4*)(r + c0), hi = *(const i32x4*)(r + c1);
      af[i] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    }
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const char* r = Bs + (wn * TN + j * 16 + frow) * ROWB;
      const i32x4 lo = *(const i32x4*)(r + c0), hi = *(const i32x4*)(r + c1);
      bfr[j] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfr[j], af[i], acc[i][j], 0,
                                                                       0, 0, 127, 0, 127);
    __builtin_amdgcn_s_setprio(0);
  };
  const int nk = p.K / ROWB;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  int cur = 0;
  for (int kt = 0; kt < nk - 1; ++kt) {
    stage(cur ^ 1, kt + 1);
    compute(cur);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur ^= 1;
  }
  compute(cur);
  constexpr int OSZ = out_size<OUT>();
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    const int64_t row = m0 + wm * TM + i * 16 + frow;
    if (row >= p.M) continue;
    char* crow = c_row<OSZ>(p, row);
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int64_t col = n0 + wn * TN + j * 16 + fq * 4;
      if (col + 3 < p.N) {
        Store4<OUT>::st(crow + col * OSZ, act4(acc[i][j], p.act));
      } else {
        const f32x4 a4 = act4(acc[i][j], p.act);
        const float v[4] = {a4.x, a4.y, a4.z, a4.w};
        for (int r = 0; r < 4; ++r)
          if (col + r < p.N) Store4<OUT>::st1(crow + (col + r) * OSZ, v[r]);
      }
    }
  }
}

// ---------------------------------------------------------------- generic fallback kernel
// Any shape / alignment / dtype (incl. f64): 64x64 tile, 4x4 per thread, f32 (f64) FMA.
template <typename T> __device__ __forceinline__ double ld_as_double(const void* p, int64_t i);
template <int DT> __device__ __forceinline__ double load_elem(const char* base, int64_t idx) {
  if constexpr (DT == DT_BF16) return (double)(float)((const __bf16*)base)[idx];
  else if constexpr (DT == DT_F16) return (double)(float)((const _Float16*)base)[idx];
  else if constexpr (DT == DT_F32) return (double)((const float*)base)[idx];
  else if constexpr (DT == DT_F64) return ((const double*)base)[idx];
  else {  // OCP e4m3fn
    const uint8_t v = ((const uint8_t*)base)[idx];
    const int s = v >> 7, e = (v >> 3) & 0xF, m = v & 7;
    double r;
    if (e == 0xF && m == 7) r = __builtin_nan("");
    else if (e == 0) r = ldexp((double)m / 8.0, -6);
    else r = ldexp(1.0 + (double)m / 8.0, e - 7);
    return s ? -r : r;
  }
}
template <int DT> __device__ __forceinline__ void store_elem(char* base, int64_t idx, double v) {
  if constexpr (DT == DT_BF16) ((__bf16*)base)[idx] = (__bf16)(float)v;
  else if constexpr (DT == DT_F16) ((_Float16*)base)[idx] = (_Float16)(float)v;
  else if constexpr (DT == DT_F32) ((float*)base)[idx] = (float)v;
  else ((double*)base)[idx] = v;
}

template <int DIN, int DOUT, typename Acc>
__global__ __launch_bounds__(256) void gemm_generic_kernel(const GemmArgs p) {
  const int tn = blockIdx.x, tm = blockIdx.y;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  Acc acc[4][4] = {};
  const char* A = (const char*)p.a;
  const char* B = (const char*)p.b;
  for (int k = 0; k < p.K; ++k) {
    Acc av[4], bv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t r = (int64_t)tm * 64 + ty * 4 + i;
      av[i] = r < p.M ? (Acc)load_elem<DIN>(A, map_row(r, p.a_grp, p.a_gstride) * p.lda + k) : 0;
      const int64_t c = (int64_t)tn * 64 + tx * 4 + i;
      bv[i] = c < p.N ? (Acc)load_elem<DIN>(B, c * p.ldb + k) : 0;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] += av[i] * bv[j];
  }
  char* C = (char*)p.c;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t r = (int64_t)tm * 64 + ty * 4 + i;
    if (r >= p.M) continue;
    const int64_t rp = map_row(r, p.c_grp, p.c_gstride) * p.ldc;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t c = (int64_t)tn * 64 + tx * 4 + j;
      if (c < p.N) store_elem<DOUT>(C, rp + c, (double)act1((float)acc[i][j], p.act));
    }
  }
}

// ---------------------------------------------------------------- dispatch
template <class Mma, int OUT, int BM, int BN, int WM, int WN, bool ILV = false>
hipError_t launch_tiled(const GemmArgs& p, hipStream_t s) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_tn_kernel<Mma, OUT, BM, BN, WM, WN, ILV>), dim3(tiles),
                     dim3(WM * WN * 64), 0, s, p);
  return hipGetLastError();
}
template <int OUT, int BM, int BN, int WM, int WN>
hipError_t launch_mx(const GemmArgs& p, hipStream_t s) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_tn_mxfp8_kernel<OUT, BM, BN, WM, WN>), dim3(tiles),
                     dim3(WM * WN * 64), 0, s, p);
  return hipGetLastError();
}

int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// t8 takes whole 256x256 tiles (flags, grouped rows, shard tables and activations allowed)
bool t8_ok(const GemmArgs& p) { return p.M % 256 == 0 && p.N % 256 == 0; }

template <class Mma, int OUT>
hipError_t launch_t8(const GemmArgs& p, hipStream_t s) {
  const int tiles = (p.M / 256) * (p.N / 256);
  hipLaunchKernelGGL((gemm_tn_t8_kernel<Mma, OUT>), dim3(tiles), dim3(512), 0, s, p);
  return hipGetLastError();
}

// Write-through C stores (CMODE 2 of pt4 / t4) whenever every C byte is within 2 GiB of p.c
// (32-bit buffer offsets); C row tables (direct store) and larger outputs keep plain nt stores.
inline bool c_fits_wt(const GemmArgs& p, int osz) {
  if (p.c_table != nullptr || p.M <= 0) return false;
  const int64_t cg = p.c_grp > 0 ? p.c_grp : p.M, cgs = p.c_gstride > 0 ? p.c_gstride : cg;
  const int64_t last_row = (int64_t)(p.M - 1) / cg * cgs + (int64_t)(p.M - 1) % cg;
  return (last_row * p.ldc + p.N) * (int64_t)osz < 0x7FFFFFF0LL;
}

template <class Mma, int OUT>
hipError_t launch_t4(const GemmArgs& p, hipStream_t s) {
  const int tiles = (p.M / 256) * (p.N / 256);
  if (c_fits_wt(p, out_size<OUT>()))
    hipLaunchKernelGGL((gemm_tn_t4_kernel<Mma, OUT, 2>), dim3(tiles), dim3(512), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_tn_t4_kernel<Mma, OUT>), dim3(tiles), dim3(512), 0, s, p);
  return hipGetLastError();
}

// pt4 needs an even number (>= 2) of K-tiles per tile (its FIRST and LAST K-tile kinds are
// distinct, its body is unrolled by buffer parity), a tile's 256 A rows contiguous (plain rows,
// grouped rows in groups of a multiple of 256, or a row-block table of such blocks: one panel
// base per tile), 32-bit panel offsets (a 256-row panel, the reach of its LDS-DMA buffer
// descriptors, stays below 1 GiB) and no fused activation (t4 carries those)
bool pt4_ok(const GemmArgs& p, int esz) {
  const int64_t nk = (int64_t)p.K * esz / 128;
  const bool a_ok = p.a_table != nullptr ? (p.shard_rows > 0 && p.shard_rows % 256 == 0)
                                         : (p.a_grp == p.M || p.a_grp % 256 == 0);
  return p.M % 256 == 0 && p.N % 256 == 0 && a_ok && p.act == ACT_NONE && nk >= 2 &&
         nk % 2 == 0 && p.lda * esz <= (1 << 22) && p.ldb * esz <= (1 << 22);
}

template <class Mma, int OUT>
hipError_t launch_pt4(const GemmArgs& p, hipStream_t s) {
  const int tiles = (p.M / 256) * (p.N / 256);
  int grid = num_cus();
  // Leave reserve_cus CUs free. A pt4 workgroup takes a CU's whole register file, so with every
  // CU holding a (spinning) tile, the copy / signal kernels that set a flag-gated GEMM's flags
  // could not be scheduled; the reserve keeps the gate deadlock-free whoever moves the data.
  // Without flags it sizes the persistent grid to a CU-masked compute stream (plans with a CU
  // split: the complement of the communication's CUs), so no workgroup waits for a free CU.
  if (p.reserve_cus > 0 && p.reserve_cus < grid) grid -= p.reserve_cus;
  GemmArgs q = p;
  q.ag_ctas = p.flags != nullptr && p.ag_ctas > 0 ? (p.ag_ctas + 7) / 8 * 8 : 0;
  // The GEMM takes ceil(tiles / gemm_ctas) rounds of tiles; every copy workgroup that leaves that
  // count unchanged is free copy bandwidth (flagship: 1024 tiles, 224 GEMM CTAs = 5 rounds, so
  // 208 GEMM + 48 copy CTAs cost the GEMM nothing more than 224 + 32).
  if (q.ag_ctas > 0 && (p.ag_mode & AG_FILL_ROUNDS)) q.ag_ctas = ag_fill_ctas(grid, q.ag_ctas, tiles);
  grid -= q.ag_ctas;
  grid = (grid / 8) * 8;  // blockIdx % 8 == XCD group for every virtual tile id
  // (A gated GEMM fed by other kernels keeps the whole num_cus - reserve_cus grid. Shrinking it
  // to the fewest workgroups that keep its tile-round count looked free, but when the transfers
  // are the bottleneck the last stage's tiles arrive at once and a smaller grid takes an extra
  // round for them: RCCL-fed s4 plan 0.202 -> 0.181 ms emulated at d = 8 without the shrink,
  // no plan slower, profiles/r04/r4_18_*.)
  const int vtiles = p.ksplit > 1 ? tiles * p.ksplit : tiles;  // (slice, tile) pairs
  if (grid > vtiles) grid = vtiles;
  if (grid < 1) grid = 1;
  // write-through stores address C from a per-tile scalar row (the tile's rows contiguous)
  const bool wt = c_fits_wt(p, out_size<OUT>()) && p.c_grp % 256 == 0;
  // A through grouped rows / a row-block table: the APAN instantiations (no C row table with them)
  const bool apan = p.a_table != nullptr || p.a_grp != p.M;
  if (p.ksplit > 1) {  // (gemm_launch routes only eligible K-splits here: plain rows, ungated)
    if (p.flags != nullptr || apan || p.c_table != nullptr || p.c_grp != p.M || !wt)
      return hipErrorNotSupported;
    if ((int64_t)p.ksplit * p.M * p.ldc * out_size<OUT>() >= 0x7FFFFFF0LL)
      return hipErrorNotSupported;
    hipLaunchKernelGGL((gemm_tn_pt4_kernel<Mma, OUT, false, 2, false, true>), dim3(grid),
                       dim3(512), 0, s, q);
    return hipGetLastError();
  }
  if (apan && p.c_table != nullptr) return hipErrorNotSupported;
  // tile_order 3 promises that the first producer's rows are never gated; only the table / grouped
  // A (APAN) gated instantiation implements that skip (OWN), so anything else is refused rather
  // than left to spin on a flag nobody raises
  if (p.flags != nullptr && p.tile_order == 3 && !apan) return hipErrorNotSupported;
  if (apan && p.flags != nullptr && wt)
    hipLaunchKernelGGL((gemm_tn_pt4_kernel<Mma, OUT, true, 2, true>), dim3(grid + q.ag_ctas),
                       dim3(512), 0, s, q);
  else if (apan && p.flags != nullptr)
    hipLaunchKernelGGL((gemm_tn_pt4_kernel<Mma, OUT, true, 0, true>), dim3(grid + q.ag_ctas),
                       dim3(512), 0, s, q);
  else if (apan && wt)
    hipLaunchKernelGGL((gemm_tn_pt4_kernel<Mma, OUT, false, 2, true>), dim3(grid), dim3(512), 0, s,
                       p);
  else if (apan)
    hipLaunchKernelGGL((gemm_tn_pt4_kernel<Mma, OUT, false, 0, true>), dim3(grid), dim3(512), 0, s,
                       p);
  else if (p.flags != nullptr && wt)
    hipLaunchKernelGGL((gemm_tn_pt4_kernel<Mma, OUT, true, 2>), dim3(grid + q.ag_ctas), dim3(512),
                       0, s, q);
  else if (p.flags != nullptr)
    hipLaunchKernelGGL((gemm_tn_pt4_kernel<Mma, OUT, true>), dim3(grid + q.ag_ctas), dim3(512), 0,
                       s, q);
  else if (p.c_table != nullptr)
    hipLaunchKernelGGL((gemm_tn_pt4_kernel<Mma, OUT, false, 1>), dim3(grid), dim3(512), 0, s, p);
  else if (wt)
    hipLaunchKernelGGL((gemm_tn_pt4_kernel<Mma, OUT, false, 2>), dim3(grid), dim3(512), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_tn_pt4_kernel<Mma, OUT, false>), dim3(grid), dim3(512), 0, s, p);
  return hipGetLastError();
}

template <class Mma, int OUT>
hipError_t launch_pt8(const GemmArgs& p, hipStream_t s) {
  const int tiles = (p.M / 256) * (p.N / 256);
  int grid = num_cus();
  // a CU split's masked compute stream: one workgroup per CU it may use (see launch_pt4)
  if (p.reserve_cus > 0 && p.reserve_cus < grid) grid -= p.reserve_cus;
  grid = (grid / 8) * 8;  // blockIdx % 8 == XCD group for every virtual tile id
  if (grid > tiles) grid = tiles;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL((gemm_tn_pt8_kernel<Mma, OUT>), dim3(grid), dim3(512), 0, s, p);
  return hipGetLastError();
}

template <class Mma, int OUT>
hipError_t launch_cfg(const GemmArgs& p, int tile, hipStream_t s) {
  switch (tile) {
    case TILE_PT8:  // persistent: no arrival flags (a block's tiles are fixed up front)
      if (t8_ok(p) && p.flags == nullptr) return launch_pt8<Mma, OUT>(p, s);
      if (t8_ok(p)) return launch_t8<Mma, OUT>(p, s);
      return launch_tiled<Mma, OUT, 256, 256, 2, 4, true>(p, s);
    case TILE_PT4:
      if (pt4_ok(p, Mma::kElem) && !(p.c_table && (p.a_table || p.a_grp != p.M)))
        return launch_pt4<Mma, OUT>(p, s);
      if (p.ksplit > 1) return hipErrorNotSupported;  // only pt4 runs (slice, tile) pairs
      if (t8_ok(p)) return launch_t4<Mma, OUT>(p, s);
      return launch_tiled<Mma, OUT, 256, 256, 2, 4, true>(p, s);
    case TILE_T4:
      if (t8_ok(p)) return launch_t4<Mma, OUT>(p, s);
      return launch_tiled<Mma, OUT, 256, 256, 2, 4, true>(p, s);
    case TILE_T8:
      if (t8_ok(p)) return launch_t8<Mma, OUT>(p, s);
      return launch_tiled<Mma, OUT, 256, 256, 2, 4, true>(p, s);
    case TILE_256x256: return launch_tiled<Mma, OUT, 256, 256, 2, 4>(p, s);
    case TILE_256x128: return launch_tiled<Mma, OUT, 256, 128, 4, 2>(p, s);
    case TILE_128x256: return launch_tiled<Mma, OUT, 128, 256, 2, 4>(p, s);
    case TILE_128x128: return launch_tiled<Mma, OUT, 128, 128, 2, 2>(p, s);
    case TILE_256x256_W4: return launch_tiled<Mma, OUT, 256, 256, 2, 2>(p, s);
    case TILE_256x128_W4: return launch_tiled<Mma, OUT, 256, 128, 2, 2>(p, s);
    case TILE_I256: return launch_tiled<Mma, OUT, 256, 256, 2, 4, true>(p, s);
    case TILE_I128: return launch_tiled<Mma, OUT, 128, 128, 2, 2, true>(p, s);
    case TILE_I256W4: return launch_tiled<Mma, OUT, 256, 256, 2, 2, true>(p, s);
    default: return hipErrorInvalidValue;  // (5, 8, 9, 13-15: retired kernel families)
  }
}
template <int OUT>
hipError_t launch_mx_cfg(const GemmArgs& p, int tile, hipStream_t s) {
  // whole 256x256 tiles: the ping-pong schedules (persistent with >= 2 tiles per CU)
  if (tile == TILE_PT4 && pt4_ok(p, 1) && !(p.c_table && (p.a_table || p.a_grp != p.M)))
    return launch_pt4<MmaMX, OUT>(p, s);
  if (p.ksplit > 1) return hipErrorNotSupported;  // only pt4 runs (slice, tile) pairs
  if ((tile == TILE_T4 || tile == TILE_PT4) && t8_ok(p)) return launch_t4<MmaMX, OUT>(p, s);
  if ((tile == TILE_T8 || tile == TILE_PT8 || tile == TILE_AUTO) && t8_ok(p)) {
    const int tiles = (p.M / 256) * (p.N / 256);
    if (tile != TILE_T8 && p.flags == nullptr && tiles >= 2 * num_cus())
      return launch_pt8<MmaMX, OUT>(p, s);
    return launch_t8<MmaMX, OUT>(p, s);
  }
  switch (tile) {
    case TILE_256x256: return launch_mx<OUT, 256, 256, 2, 4>(p, s);
    case TILE_256x128: return launch_mx<OUT, 256, 128, 4, 2>(p, s);
    case TILE_128x256: return launch_mx<OUT, 128, 256, 2, 4>(p, s);
    case TILE_128x128: return launch_mx<OUT, 128, 128, 2, 2>(p, s);
    case TILE_256x256_W4: return launch_mx<OUT, 256, 256, 2, 2>(p, s);
    case TILE_I256: return launch_mx<OUT, 256, 256, 2, 4>(p, s);
    case TILE_I128: return launch_mx<OUT, 128, 128, 2, 2>(p, s);
    case TILE_I256W4: return launch_mx<OUT, 256, 256, 2, 2>(p, s);
    case TILE_T8: case TILE_PT8: case TILE_T4: case TILE_PT4:
      return launch_mx<OUT, 256, 256, 2, 4>(p, s);
    case TILE_256x128_W4: return launch_mx<OUT, 256, 128, 2, 2>(p, s);
    default: return hipErrorInvalidValue;  // (5, 8, 9, 13-15: retired kernel families)
  }
}

template <int DIN, int DOUT>
hipError_t launch_generic_t(const GemmArgs& p, hipStream_t s) {
  dim3 grid((p.N + 63) / 64, (p.M + 63) / 64);
  if constexpr (DIN == DT_F64)
    hipLaunchKernelGGL((gemm_generic_kernel<DIN, DOUT, double>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_generic_kernel<DIN, DOUT, float>), grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace
}  // namespace ddlb
