// Small data-movement / synchronisation kernels used by the plan executor.
//
//  * reduce_sum: dst = sum_j src_j (up to 16 sources, any of them peer memory over xGMI), f32
//    accumulation, one rounding — the fused "sum d partial tiles -> output" of the p2p
//    reduce-scatter (SURVEY.md §2.4 "Reductions inside RS").
//  * copy: CU-driven 16-byte vector copy (the `kernel` protocol; stands in for NVLS multimem,
//    which MI355X does not have). Reads/writes may be peer pointers.
//  * signal / wait: cross-process flags in symmetric memory. Release stores at system scope,
//    bounded relaxed polling, acquire at system scope after the match (cdna guide §6 G16).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <stdlib.h>

#include "kernels.h"

namespace ddlb {
namespace {

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;

template <int DT> struct V8;  // 16-byte vector of the element type, widened to f32
template <> struct V8<0> {    // f32: 4 elements per 16 B
  static constexpr int N = 4;
  static __device__ __forceinline__ void load(const void* p, float* o) {
    const f32x4 v = *(const f32x4*)p;
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
  static __device__ __forceinline__ void store(void* p, const float* o) {
    *(f32x4*)p = f32x4{o[0], o[1], o[2], o[3]};
  }
};
template <> struct V8<1> {  // f16
  static constexpr int N = 8;
  static __device__ __forceinline__ void load(const void* p, float* o) {
    const f16x8 v = *(const f16x8*)p;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (float)v[i];
  }
  static __device__ __forceinline__ void store(void* p, const float* o) {
    f16x8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (_Float16)o[i];
    *(f16x8*)p = v;
  }
};
template <> struct V8<2> {  // bf16
  static constexpr int N = 8;
  static __device__ __forceinline__ void load(const void* p, float* o) {
    const bf16x8 v = *(const bf16x8*)p;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (float)v[i];
  }
  static __device__ __forceinline__ void store(void* p, const float* o) {
    bf16x8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (__bf16)o[i];
    *(bf16x8*)p = v;
  }
};

template <int DT>
__device__ __forceinline__ float load1(const void* p, int64_t i) {
  if constexpr (DT == 0) return ((const float*)p)[i];
  else if constexpr (DT == 1) return (float)((const _Float16*)p)[i];
  else return (float)((const __bf16*)p)[i];
}
template <int DT>
__device__ __forceinline__ void store1(void* p, int64_t i, float v) {
  if constexpr (DT == 0) ((float*)p)[i] = v;
  else if constexpr (DT == 1) ((_Float16*)p)[i] = (_Float16)v;
  else ((__bf16*)p)[i] = (__bf16)v;
}

template <int DT>
__global__ __launch_bounds__(256) void reduce_sum_kernel(ReduceArgs a) {
  using V = V8<DT>;
  const int64_t nvec = a.count / V::N;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float acc[V::N], t[V::N];
    V::load((const char*)a.src[0] + v * 16, acc);
    for (int s = 1; s < a.nsrc; ++s) {
      V::load((const char*)a.src[s] + v * 16, t);
#pragma unroll
      for (int i = 0; i < V::N; ++i) acc[i] += t[i];
    }
    V::store((char*)a.dst + v * 16, acc);
  }
  const int64_t tail0 = nvec * V::N;
  for (int64_t i = tail0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.count;
       i += stride) {
    float acc = 0.f;
    for (int s = 0; s < a.nsrc; ++s) acc += load1<DT>(a.src[s], i);
    store1<DT>(a.dst, i, acc);
  }
}

// Fixed source count: all NS 16-byte loads of a lane are issued before the first add, so NS
// requests per lane are in flight at once (the runtime-count loop above waits on each load before
// issuing the next). Matters when the sources are peers' buffers read over xGMI, where latency
// is several microseconds. Loads and the store are non-temporal (streamed once). Summation order is src[0] + src[1] + ... as above (bitwise equal).
template <int DT, int NS>
__global__ __launch_bounds__(256) void reduce_sum_fixed_kernel(ReduceArgs a) {
  using V = V8<DT>;
  const int64_t nvec = a.count / V::N;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    u32x4 raw[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s)
      raw[s] = __builtin_nontemporal_load((const u32x4*)((const char*)a.src[s] + v * 16));
    float acc[V::N], t[V::N];
    V::load(&raw[0], acc);
#pragma unroll
    for (int s = 1; s < NS; ++s) {
      V::load(&raw[s], t);
#pragma unroll
      for (int i = 0; i < V::N; ++i) acc[i] += t[i];
    }
    u32x4 o;
    V::store(&o, acc);
    __builtin_nontemporal_store(o, (u32x4*)((char*)a.dst + v * 16));  // streamed, read by no one here
  }
  const int64_t tail0 = nvec * V::N;
  for (int64_t i = tail0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.count;
       i += stride) {
    float acc = 0.f;
    for (int s = 0; s < NS; ++s) acc += load1<DT>(a.src[s], i);
    store1<DT>(a.dst, i, acc);
  }
}

// f32 sources -> a 16-bit destination (f16 / bf16): the K-split GEMM's f32 partials summed and
// rounded ONCE. A lane takes 8 elements: 32 B of every source (NS > 0: all loads issued before
// the first add; NS == 0: a.nsrc sources, one at a time), 16 B out. Same source order.
template <int DDT, int NS>
__global__ __launch_bounds__(256) void reduce_f32_to_kernel(ReduceArgs a) {
  using V = V8<DDT>;
  static_assert(V::N == 8, "16-bit destinations only");
  const int64_t nvec = a.count / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float acc[8];
    if constexpr (NS > 0) {
      f32x4 raw[NS][2];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const f32x4* p = (const f32x4*)((const char*)a.src[s] + v * 32);
        raw[s][0] = __builtin_nontemporal_load(p);
        raw[s][1] = __builtin_nontemporal_load(p + 1);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) { acc[i] = raw[0][0][i]; acc[4 + i] = raw[0][1][i]; }
#pragma unroll
      for (int s = 1; s < NS; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) { acc[i] += raw[s][0][i]; acc[4 + i] += raw[s][1][i]; }
    } else {
      for (int i = 0; i < 8; ++i) acc[i] = 0.f;
      for (int s = 0; s < a.nsrc; ++s) {
        const f32x4* p = (const f32x4*)((const char*)a.src[s] + v * 32);
        const f32x4 lo = __builtin_nontemporal_load(p), hi = __builtin_nontemporal_load(p + 1);
        if (s == 0) {
          for (int i = 0; i < 4; ++i) { acc[i] = lo[i]; acc[4 + i] = hi[i]; }
        } else {
          for (int i = 0; i < 4; ++i) { acc[i] += lo[i]; acc[4 + i] += hi[i]; }
        }
      }
    }
    u32x4 o;
    V::store(&o, acc);
    __builtin_nontemporal_store(o, (u32x4*)((char*)a.dst + v * 16));
  }
  const int ns = NS > 0 ? NS : a.nsrc;
  for (int64_t i = nvec * 8 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.count;
       i += stride) {
    float acc = load1<0>(a.src[0], i);
    for (int s = 1; s < ns; ++s) acc += load1<0>(a.src[s], i);
    store1<DDT>(a.dst, i, acc);
  }
}

// Blocks are dealt round-robin to the segments (one segment = one peer = one xGMI link in the
// IPC all-gathers), so every link carries traffic at once; the blocks of a segment grid-stride
// over it with U x 16 B in flight per lane (8 by default: a peer read over xGMI has several times
// the latency of local HBM, and bytes in flight per CU are what bound a latency-bound pull).
// (Walking the segments one after another would keep a single link busy at a time: d-1 times the
// transfer time of a full-mesh exchange.)
template <bool NT>  // NT: non-temporal source loads (each source byte is read exactly once)
__device__ __forceinline__ u32x4 copy_ld(const char* p) {
  if constexpr (NT)
    return __builtin_nontemporal_load((const u32x4*)p);
  else
    return *(const u32x4*)p;
}

template <bool NT, int U>
__global__ __launch_bounds__(256) void copy_kernel(CopyArgs a) {
  const int nseg = a.nseg;
  const int seg = (int)blockIdx.x % nseg;
  const int nb = ((int)gridDim.x - seg + nseg - 1) / nseg;  // blocks serving this segment
  const int64_t stride = (int64_t)nb * blockDim.x;
  const int64_t t0 = (int64_t)((int)blockIdx.x / nseg) * blockDim.x + threadIdx.x;
  const char* src = (const char*)a.src[seg];
  char* dst = (char*)a.dst[seg];
  const int64_t bytes = a.bytes[seg];
  const int64_t nvec = bytes / 16;
  int64_t v = t0;
  for (; v + (U - 1) * stride < nvec; v += U * stride) {
    u32x4 x[U];
#pragma unroll
    for (int i = 0; i < U; ++i) x[i] = copy_ld<NT>(src + (v + i * stride) * 16);
#pragma unroll
    for (int i = 0; i < U; ++i) *(u32x4*)(dst + (v + i * stride) * 16) = x[i];
  }
  for (; v < nvec; v += stride) *(u32x4*)(dst + v * 16) = copy_ld<NT>(src + v * 16);
  for (int64_t b = nvec * 16 + t0; b < bytes; b += stride) dst[b] = src[b];
}

__global__ void signal_kernel(SignalArgs a) {
  const int i = threadIdx.x;
  if (i < a.n) {
    const unsigned v = a.epoch_ptr ? (unsigned)((int)*a.epoch_ptr + a.delta) : a.value;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    __hip_atomic_store(a.ptr[i], v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void wait_kernel(WaitArgs a) {
  if (threadIdx.x != 0) return;
  const int want = a.epoch_ptr ? (int)*a.epoch_ptr + a.delta : (int)a.value;
  if (want <= 0) return;  // nothing to wait for before the first epoch
  for (int i = 0; i < a.n; ++i) {
    unsigned spins = 0;
    while (__hip_atomic_load(a.ptr[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) <
           (unsigned)want) {
      __builtin_amdgcn_s_sleep(4);
      if (++spins > (1u << 27)) {  // bounded: report and drain instead of hanging the GPU
        if (a.timeout_word) atomicOr(a.timeout_word, 2u);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

__global__ void bump_signal_kernel(BumpSignalArgs a) {
  __shared__ unsigned e;
  if (threadIdx.x == 0) {
    e = *a.epoch + 1;
    *a.epoch = e;
  }
  __syncthreads();
  const int i = threadIdx.x;
  if (i < a.n) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    __hip_atomic_store(a.ptr[i], (unsigned)((int)e + a.delta[i]), __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void epoch_bump_kernel(unsigned* epoch) {
  if (threadIdx.x == 0) *epoch += 1;
}

// CU holder: each workgroup takes a whole CU the way the flag-gated persistent pt4 GEMM does (512
// threads at 256 VGPRs = the full register file, plus all 160 KB of LDS), counts itself resident
// in *arrived (host-coherent memory) and spins, bounded, until the host sets *go.
__global__ __launch_bounds__(512, 1) void hold_cus_kernel(HoldArgs a) {
  __shared__ char pad[160 * 1024];
  asm volatile("" ::: "v255");  // a 256-VGPR allocation, as the gated GEMM's
  pad[threadIdx.x * 320] = 1;   // touched across all 160 KB, so all of it is allocated
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(a.arrived, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // bounded in wall time (s_memrealtime: 100 MHz), not in polls: a poll of host memory costs
    // a PCIe round trip, so a poll count says little about how long a holder can stay
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(a.go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
      __builtin_amdgcn_s_sleep(32);
      if (__builtin_amdgcn_s_memrealtime() - t0 > a.max_ticks) {  // never outlives a lost host
        atomicOr(a.timeout_word, 4u);
        break;
      }
    }
  }
  __syncthreads();
  if (pad[threadIdx.x * 320] != 1) atomicOr(a.timeout_word, 8u);  // (keeps the LDS array)
}

int grid_for(int64_t work_items) {
  int64_t g = (work_items + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

hipError_t reduce_sum_launch(const ReduceArgs& a, int dtype, hipStream_t s, int src_dtype) {
  if (a.nsrc < 1 || a.nsrc > kMaxReduceSrc || a.count <= 0) return hipErrorInvalidValue;
  for (int i = 0; i < a.nsrc; ++i)
    if ((uintptr_t)a.src[i] & 15) return hipErrorInvalidValue;
  if ((uintptr_t)a.dst & 15) return hipErrorInvalidValue;
  if (src_dtype >= 0 && src_dtype != dtype) {  // f32 partials -> f16 / bf16, one rounding
    if (src_dtype != 0 || (dtype != 1 && dtype != 2)) return hipErrorInvalidValue;
    const int g = grid_for(a.count / 8 + 1);
#define DDLB_RF_CASE(NS)                                                                    \
  case NS:                                                                                  \
    if (dtype == 1) hipLaunchKernelGGL((reduce_f32_to_kernel<1, NS>), dim3(g), dim3(256), 0, s, a); \
    else hipLaunchKernelGGL((reduce_f32_to_kernel<2, NS>), dim3(g), dim3(256), 0, s, a);    \
    break;
    switch (a.nsrc >= 2 && a.nsrc <= 8 ? a.nsrc : 0) {
      DDLB_RF_CASE(0) DDLB_RF_CASE(2) DDLB_RF_CASE(3) DDLB_RF_CASE(4) DDLB_RF_CASE(5)
      DDLB_RF_CASE(6) DDLB_RF_CASE(7) DDLB_RF_CASE(8)
    }
#undef DDLB_RF_CASE
    return hipGetLastError();
  }
  const int per = dtype == 0 ? 4 : 8;
  const int g = grid_for(a.count / per + 1);
  static const bool generic = getenv("DDLB_REDUCE_GENERIC") != nullptr;  // A/B knob (benches)
  if (!generic && a.nsrc >= 2 && a.nsrc <= 8 && dtype >= 0 && dtype <= 2) {
#define DDLB_RS_CASE(NS)                                                                    \
  case NS:                                                                                  \
    if (dtype == 0) hipLaunchKernelGGL((reduce_sum_fixed_kernel<0, NS>), dim3(g), dim3(256), 0, s, a); \
    else if (dtype == 1) hipLaunchKernelGGL((reduce_sum_fixed_kernel<1, NS>), dim3(g), dim3(256), 0, s, a); \
    else hipLaunchKernelGGL((reduce_sum_fixed_kernel<2, NS>), dim3(g), dim3(256), 0, s, a); \
    break;
    switch (a.nsrc) {
      DDLB_RS_CASE(2) DDLB_RS_CASE(3) DDLB_RS_CASE(4) DDLB_RS_CASE(5)
      DDLB_RS_CASE(6) DDLB_RS_CASE(7) DDLB_RS_CASE(8)
    }
#undef DDLB_RS_CASE
    return hipGetLastError();
  }
  switch (dtype) {
    case 0: hipLaunchKernelGGL(reduce_sum_kernel<0>, dim3(g), dim3(256), 0, s, a); break;
    case 1: hipLaunchKernelGGL(reduce_sum_kernel<1>, dim3(g), dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL(reduce_sum_kernel<2>, dim3(g), dim3(256), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t copy_launch(const CopyArgs& a, int max_blocks, hipStream_t s) {
  if (a.nseg < 1 || a.nseg > kMaxCopySeg) return hipErrorInvalidValue;
  int64_t total = 0;
  for (int i = 0; i < a.nseg; ++i) {
    if (((uintptr_t)a.src[i] | (uintptr_t)a.dst[i]) & 15) return hipErrorInvalidValue;
    total += a.bytes[i];
  }
  int g = grid_for(total / 64 + 1);
  if (max_blocks > 0 && g > max_blocks) g = max_blocks;
  // at least one block per segment, and a whole number of blocks per segment
  g = g < a.nseg ? a.nseg : (g / a.nseg) * a.nseg;
  // Plain loads by default: non-temporal source loads measured slower on HBM (7 x 16 MiB:
  // 52 vs 34 us at 128 blocks, 36 vs 35 at 512; profiles/r01/s3/copy_ab_nt.txt). A/B knob kept.
  // DDLB_COPY_U=4: the earlier 4 loads in flight per lane (A/B knob).
  static const bool nt = getenv("DDLB_COPY_NT") != nullptr;
  static const bool u4 = getenv("DDLB_COPY_U") != nullptr && atoi(getenv("DDLB_COPY_U")) == 4;
  if (nt && u4) hipLaunchKernelGGL((copy_kernel<true, 4>), dim3(g), dim3(256), 0, s, a);
  else if (nt) hipLaunchKernelGGL((copy_kernel<true, 8>), dim3(g), dim3(256), 0, s, a);
  else if (u4) hipLaunchKernelGGL((copy_kernel<false, 4>), dim3(g), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((copy_kernel<false, 8>), dim3(g), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t signal_launch(const SignalArgs& a, hipStream_t s) {
  if (a.n < 1 || a.n > kMaxSignal) return hipErrorInvalidValue;
  hipLaunchKernelGGL(signal_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t wait_launch(const WaitArgs& a, hipStream_t s) {
  if (a.n < 1 || a.n > kMaxSignal) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wait_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t bump_signal_launch(const BumpSignalArgs& a, hipStream_t s) {
  if (a.epoch == nullptr || a.n < 0 || a.n > kMaxPrologue) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bump_signal_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t hold_cus_launch(const HoldArgs& a, int nwg, hipStream_t s) {
  if (nwg < 1 || a.arrived == nullptr || a.go == nullptr || a.timeout_word == nullptr)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(hold_cus_kernel, dim3(nwg), dim3(512), 0, s, a);
  return hipGetLastError();
}

hipError_t epoch_bump_launch(unsigned* epoch, hipStream_t s) {
  hipLaunchKernelGGL(epoch_bump_kernel, dim3(1), dim3(64), 0, s, epoch);
  return hipGetLastError();
}

}  // namespace ddlb
