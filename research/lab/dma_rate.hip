// LDS-DMA rate microbenchmark (lab, not part of the extension): how many bytes per clock per CU
// can global_load_lds_dwordx4 (1 KiB per wave-instruction) move, as a function of the number of
// instructions each wave keeps in flight, from an L2-resident source and from an HBM-streamed one?
// Tells whether the GEMM's LDS-DMA path is bounded by the per-CU vector-memory path or by latency
// x bytes in flight.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 research/lab/dma_rate.hip -o research/lab/bin/dma_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Each wave streams `iters` 1-KiB LDS-DMA pieces from src (wrapping inside `span` bytes, offset
// per block so blocks do not share lines unless span is small) into its own 8 KiB LDS ring,
// keeping INFLIGHT pieces outstanding. STORE: each piece is instead a 1-KiB global store.
// BUF: the same through a buffer resource (wave-uniform descriptor + 32-bit per-lane offset)
template <int INFLIGHT, bool STORE, bool BUF = false>
__global__ __launch_bounds__(512) void dma_kernel(const char* src, char* dst, int64_t span,
                                                  int iters, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(1024))) char smem[8 * 8192];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  char* ring = smem + wave * 8192;
  const int64_t base = ((int64_t)blockIdx.x * 8 + wave) * (int64_t)iters * 1024;  // disjoint per wave
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  int64_t off = base;
  for (int i = 0; i < iters; ++i) {
    // L2-resident mode: waves start at different 1 KiB pieces of the span (no hot spot)
    // (span is a power of two: a mask, not a 64-bit modulo, which would bound the loop itself)
    const int64_t o = (off + ((int64_t)blockIdx.x * 8 + wave) * 37 * 1024) & (span - 1);
    if constexpr (BUF) {
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
          STORE ? (void*)dst : (void*)src, 0, 0x7FFFFFF0, 0x00020000);
      if constexpr (STORE) {
        typedef __attribute__((ext_vector_type(4))) int i32x4;
        const i32x4 v = {i, 0, 0, lane};
        __builtin_amdgcn_raw_buffer_store_b128(v, r, (unsigned)o + lane * 16, 0, 0);
      } else {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)(ring + (i & 7) * 1024), 16,
                                                 (unsigned)o + lane * 16, 0, 0, 0);
      }
    } else if constexpr (STORE) {
      uint4 v = {(unsigned)i, 0u, 0u, (unsigned)lane};
      *(uint4*)(dst + o + lane * 16) = v;
    } else {
      __builtin_amdgcn_global_load_lds((const GLB_AS void*)(src + o + lane * 16),
                                       (LDS_AS void*)(ring + (i & 7) * 1024), 16, 0, 0);
    }
    wait_vm<INFLIGHT>();
    off += 1024;
  }
  wait_vm<0>();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0 && wave == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int INFLIGHT, bool STORE, bool BUF = false>
void run(const char* tag, const char* src, char* dst, int64_t span, int nblk, int iters,
         unsigned long long* cyc) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((dma_kernel<INFLIGHT, STORE, BUF>), dim3(nblk), dim3(512), 0, 0, src, dst, span,
                     iters, cyc);
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL((dma_kernel<INFLIGHT, STORE, BUF>), dim3(nblk), dim3(512), 0, 0, src, dst,
                       span, iters, cyc);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 5;
  unsigned long long* h = (unsigned long long*)malloc(nblk * 8);
  CHECK(hipMemcpy(h, cyc, nblk * 8, hipMemcpyDeviceToHost));
  double mc = 0;
  for (int i = 0; i < nblk; ++i) mc += (double)h[i];
  mc /= nblk;
  free(h);
  const double bytes = (double)nblk * 8 * iters * 1024;
  printf("%-28s inflight %2d: %8.3f ms  %7.2f TB/s  %6.1f B/clk/CU (in-kernel clocks, mean over blocks)\n",
         tag, INFLIGHT, ms, bytes / (ms * 1e-3) / 1e12, bytes / nblk / mc);
}

int main() {
  int dev = 0, ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int64_t big = 2ll << 30;  // 2 GiB: streamed from HBM
  char *src, *dst;
  CHECK(hipMalloc(&src, big));
  CHECK(hipMalloc(&dst, big));
  CHECK(hipMemset(src, 1, big));
  unsigned long long* cyc;
  CHECK(hipMalloc(&cyc, ncu * 8 * sizeof(unsigned long long)));
  const int iters = 4096;  // 4 MiB per wave, 32 MiB per CU
  printf("%d CUs, 8 waves per CU, 1 KiB per instruction\n", ncu);
  const int64_t l2 = 1 << 20;  // 1 MiB: L2-resident
  run<1, false>("LDS-DMA, L2-resident", src, dst, l2, ncu, iters, cyc);
  run<2, false>("LDS-DMA, L2-resident", src, dst, l2, ncu, iters, cyc);
  run<4, false>("LDS-DMA, L2-resident", src, dst, l2, ncu, iters, cyc);
  run<8, false>("LDS-DMA, L2-resident", src, dst, l2, ncu, iters, cyc);
  run<16, false>("LDS-DMA, L2-resident", src, dst, l2, ncu, iters, cyc);
  run<2, false>("LDS-DMA, HBM-streamed", src, dst, big, ncu, iters / 8, cyc);
  run<4, false>("LDS-DMA, HBM-streamed", src, dst, big, ncu, iters / 8, cyc);
  run<8, false>("LDS-DMA, HBM-streamed", src, dst, big, ncu, iters / 8, cyc);
  run<16, false>("LDS-DMA, HBM-streamed", src, dst, big, ncu, iters / 8, cyc);
  run<4, true>("store, L2-resident", src, dst, l2, ncu, iters, cyc);
  run<16, true>("store, L2-resident", src, dst, l2, ncu, iters, cyc);
  run<16, true>("store, HBM-streamed", src, dst, big, ncu, iters / 8, cyc);
  run<2, false, true>("buffer LDS-DMA, L2-resident", src, dst, l2, ncu, iters, cyc);
  run<8, false, true>("buffer LDS-DMA, L2-resident", src, dst, l2, ncu, iters, cyc);
  run<4, true, true>("buffer store, L2-resident", src, dst, l2, ncu, iters, cyc);
  run<16, true, true>("buffer store, L2-resident", src, dst, l2, ncu, iters, cyc);
  run<16, true, true>("buffer store, HBM-streamed", src, dst, big, ncu, iters / 8, cyc);
  return 0;
}
