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
// Signal / wait values: ``value``, or — when ``epoch_ptr`` is set (hipGraph replay, where no
// host-side value can change between replays) — ``*epoch_ptr + delta`` read on the device.
struct SignalArgs {          // *ptr[i] = value (system-scope release), i < n
  unsigned* ptr[kMaxSignal] = {};
  unsigned value = 0;
  int n = 0;
  const unsigned* epoch_ptr = nullptr;
  int delta = 0;
};
struct WaitArgs {            // spin until *ptr[i] >= value for all i (bounded); value <= 0: no-op
  unsigned* ptr[kMaxSignal] = {};
  unsigned value = 0;
  int n = 0;
  unsigned* timeout_word = nullptr;
  const unsigned* epoch_ptr = nullptr;
  int delta = 0;
};

// src_dtype < 0: the sources have the destination's dtype; 0 (f32) with a f16 / bf16 destination:
// f32 partials summed and rounded once
hipError_t reduce_sum_launch(const ReduceArgs& a, int dtype, hipStream_t s, int src_dtype = -1);
hipError_t copy_launch(const CopyArgs& a, int max_blocks, hipStream_t s);
hipError_t signal_launch(const SignalArgs& a, hipStream_t s);
hipError_t wait_launch(const WaitArgs& a, hipStream_t s);
// *epoch += 1 (one lane): the device-side run counter of a graph-replayed plan.
hipError_t epoch_bump_launch(unsigned* epoch, hipStream_t s);
// hipGraph prologue: ++*epoch, then *ptr[i] = new epoch + delta[i] (system-scope release) — the
// run-counter bump and the plan's leading signals in ONE launch instead of 1 + k.
constexpr int kMaxPrologue = 32;
struct BumpSignalArgs {
  unsigned* epoch = nullptr;
  unsigned* ptr[kMaxPrologue] = {};
  int delta[kMaxPrologue] = {};
  int n = 0;
};
hipError_t bump_signal_launch(const BumpSignalArgs& a, hipStream_t s);
// CU holder (preflight ``rccl_cap``): ``nwg`` workgroups that each occupy a whole CU as the
// flag-gated persistent GEMM does (full register file + LDS), count themselves in *arrived and
// spin until *go != 0 (bounded: max_ticks of the 100 MHz s_memrealtime clock; then timeout bit
// 4 in *timeout_word).
struct HoldArgs {
  unsigned* arrived = nullptr;
  const unsigned* go = nullptr;
  unsigned* timeout_word = nullptr;
  uint64_t max_ticks = 1000000000ull;  // 10 s
};
hipError_t hold_cus_launch(const HoldArgs& a, int nwg, hipStream_t s);

}  // namespace ddlb
