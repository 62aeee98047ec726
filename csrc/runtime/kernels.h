// Utility kernels for the plan executor (csrc/runtime/kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ddlb {

constexpr int kMaxReduceSrc = 16;
constexpr int kMaxCopySeg = 8;
constexpr int kMaxSignal = 16;

struct ReduceArgs {          // dst[i] = sum_s src[s][i]  (dtype 0 f32, 1 f16, 2 bf16)
  void* dst = nullptr;
  const void* src[kMaxReduceSrc] = {};
  int nsrc = 0;
  int64_t count = 0;
};
struct CopyArgs {            // nseg independent byte copies, 16-byte aligned
  void* dst[kMaxCopySeg] = {};
  const void* src[kMaxCopySeg] = {};
  int64_t bytes[kMaxCopySeg] = {};
  int nseg = 0;
};
struct SignalArgs {          // *ptr[i] = value (system-scope release), i < n
  unsigned* ptr[kMaxSignal] = {};
  unsigned value = 0;
  int n = 0;
};
struct WaitArgs {            // spin until *ptr[i] >= value for all i (bounded)
  unsigned* ptr[kMaxSignal] = {};
  unsigned value = 0;
  int n = 0;
  unsigned* timeout_word = nullptr;
};

hipError_t reduce_sum_launch(const ReduceArgs& a, int dtype, hipStream_t s);
hipError_t copy_launch(const CopyArgs& a, int max_blocks, hipStream_t s);
hipError_t signal_launch(const SignalArgs& a, hipStream_t s);
hipError_t wait_launch(const WaitArgs& a, hipStream_t s);

}  // namespace ddlb
