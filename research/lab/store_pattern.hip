// Store-pattern microbenchmark: does a 16-byte-per-lane write-through store stream run faster when
// each instruction covers whole 128-byte lines (8 rows x 128 B) than when it covers half lines
// (16 rows x 64 B, the pt4 bf16 epilogue's pattern)? A 65536 x 1024 bf16 matrix (128 MB, the flagship's C) written by
// 256 x 512-thread workgroups, each wave a 16 x 64 block at a time.
//
//   hipcc --offload-arch=gfx950 -O3 -o research/lab/bin/store_pattern research/lab/store_pattern.hip
//   research/lab/bin/store_pattern
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

constexpr int M = 65536, N = 1024, ROWB = N * 2;

// PAT 0: half lines (lane = row frow (16) x 16-B chunk fq (4) of a 32-col quadrant; two
//        instructions: quadrants 0 / 1)
// PAT 1: whole lines (lane = row r (8) x chunk c (8) of the 64-col block; two instructions: rows
//        0-7 / 8-15)
template <int PAT, int AUX>
__global__ __launch_bounds__(512) void store_kernel(char* c, int reps) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwaves = gridDim.x * 8;
  const int gw = blockIdx.x * 8 + wave;
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(c, 0, 0x7FFFFFF0, 0x00020000);
  const int nblk = (M / 16) * (N / 64);  // 16 x 64 blocks
  u32x4 v = {(unsigned)lane, 1u, 2u, 3u};
  for (int r = 0; r < reps; ++r) {
    for (int b = gw; b < nblk; b += nwaves) {
      const int br = (b / (N / 64)) * 16, bc = (b % (N / 64)) * 64;
      const unsigned base = (unsigned)(br * ROWB + bc * 2);
      unsigned o0, o1;
      if constexpr (PAT == 0) {
        const int frow = lane & 15, fq = lane >> 4;
        o0 = base + frow * ROWB + fq * 16;
        o1 = o0 + 64;
      } else {
        const int rr = lane >> 3, cc = lane & 7;
        o0 = base + rr * ROWB + cc * 16;
        o1 = o0 + 8 * ROWB;
      }
      __builtin_amdgcn_raw_buffer_store_b128(v, rc, o0, 0, AUX);
      __builtin_amdgcn_raw_buffer_store_b128(v, rc, o1, 0, AUX);
    }
  }
}

template <int PAT, int AUX>
float run(char* c, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((store_kernel<PAT, AUX>), dim3(256), dim3(512), 0, 0, c, 1);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a, 0));
  hipLaunchKernelGGL((store_kernel<PAT, AUX>), dim3(256), dim3(512), 0, 0, c, reps);
  CHECK(hipEventRecord(b, 0));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms / reps;
}

int main() {
  char* c;
  CHECK(hipMalloc(&c, (size_t)M * ROWB));
  const int reps = 20;
  const double gb = (double)M * ROWB / 1e9;
  for (int round = 0; round < 3; ++round) {
    const float t0 = run<0, 18>(c, reps), t1 = run<1, 18>(c, reps);
    const float t2 = run<0, 2>(c, reps), t3 = run<1, 2>(c, reps);
    printf("round %d  sc1|nt: half lines %.1f us (%.2f TB/s)  whole lines %.1f us (%.2f TB/s)   "
           "nt: half %.1f us  whole %.1f us\n",
           round, t0 * 1e3, gb / t0, t1 * 1e3, gb / t1, t2 * 1e3, t3 * 1e3);
  }
  CHECK(hipFree(c));
  return 0;
}
