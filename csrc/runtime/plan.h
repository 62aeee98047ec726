// Plan executor: a tiny host IR for distributed-GEMM schedules, executed natively.
//
// The reference lowers its pipelines through nvFuser's MultiDeviceExecutor / host IR
// (ddlb/primitives/TPColumnwise/fuser.py:247-257). Here Python (ddlb_amd/parallel/plan.py) builds a
// flat list of ops once at construction; every run() is ONE call into this executor, which
// enqueues GEMM kernels, RCCL collectives, copy-engine transfers, cross-process signals and
// event edges on a fixed set of HIP streams. Stream 0 is the caller's stream: the executor forks
// every other stream from it at the start and joins them back at the end, so the plan is
// ordered with surrounding torch work and a device synchronize covers all of it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

#include "../comm/comm.h"
#include "../gemm/gemm.h"
#include "plan_ir.h"

namespace ddlb {

// Op layout and kinds: plan_ir.h (the host-only decoder / validator this executor runs on).
// hipMemcpyBatchAsync, resolved at run time (dlsym): the HIP runtime torch ships (7.0) predates
// it, so a batch falls back to one hipMemcpyAsync per segment on the same stream there.
bool copy_batch_api_available();
std::string copy_batch_status();  // what copy_batch did so far (see plan.cpp)
hipError_t copy_batch(void** dst, void** src, size_t* bytes, size_t n, hipStream_t s);
// Host stack trace on SIGSEGV / SIGABRT / SIGBUS (glibc backtrace to stderr, then the default
// action): a native frame list for crashes inside the HIP runtime without attaching a debugger.
void install_crash_handler();

class PlanExecutor {
 public:
  PlanExecutor(int device, int nstreams, int nevents, const std::vector<int>& priorities);
  ~PlanExecutor();
  void load(const std::vector<int64_t>& ops);
  void set_comm(RcclComm* comm) { comm_ = comm; }
  // CU budget of the communication: the side streams (RCCL / copy kernels /
  // flag kernels) are created with hipExtStreamCreateWithCUMask on `comm_cus` CUs, and the
  // plan's stream-0 ops run on a private compute stream masked to the complement (forked from
  // and joined back into the caller's stream). 0 = unmasked. Call before the first run().
  void set_cu_split(int comm_cus);
  int cu_split() const { return comm_cus_; }
  // (index, hipStreamGetFlags, hipStreamGetPriority) of every side stream and, with a CU split,
  // of the masked compute stream (index -1): what HIP actually gave the streams (a CU-masked
  // stream is created without flags / priority arguments)
  std::vector<std::vector<int>> stream_info() const;
  // Stage-level tracing: while on, every op's enqueue is wrapped in a roctx range named by
  // `labels` (e.g. "gemm s3", "copy p2 b1"), so `rocprofv3 --marker-trace --kernel-rename`
  // splits a pipeline run into its stages. roctx is loaded lazily (no link dependency).
  void set_trace(bool on, const std::vector<std::string>& labels);
  // Enqueue the whole plan behind `main_stream`; returns the epoch used (1, 2, ...).
  unsigned run(uintptr_t main_stream);
  unsigned epoch() const { return epoch_; }
  int nops() const { return (int)(ops_.size() / kOpWords); }
  uintptr_t timeout_word() const { return (uintptr_t)d_timeout_; }
  unsigned read_timeout();  // synchronous; 0 = healthy
  uintptr_t stream(int i) const { return (uintptr_t)streams_.at(i); }
  // hipGraph mode: the plan is captured once (on a private stream) and replayed with one
  // hipGraphLaunch behind the caller's stream (host cost of a run: one launch instead of one
  // HIP / RCCL call per op). Epoch-dependent ops read a device-side run counter in this mode.
  void enable_graph(bool on);
  bool graph_enabled() const { return graph_on_; }
  bool graph_capturable() const;
  // Per-op GPU timeline (observability): while on, run() records a timing event on the caller's
  // stream before the fork and one on each op's stream right after the op. timeline() waits
  // for the last run and returns, per op, the ms from the fork to the end of that op on its
  // stream (ops with nothing to enqueue report their stream's previous end). Not with graphs.
  void set_timeline(bool on);
  std::vector<float> timeline();
  // Host-side cost of enqueueing each op in the last run (us), recorded while the timeline is on.
  std::vector<float> host_times() const { return host_us_; }

 private:
  void exec(const int64_t* op, hipStream_t main);
  GemmArgs gemm_args(const int64_t* op) const;
  void enqueue(hipStream_t main);
  bool any_side_ = false;
  bool graph_on_ = false;
  hipStream_t cap_stream_ = nullptr;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t graph_exec_ = nullptr;
  // OP_COPY_BATCH without hipMemcpyBatchAsync (eager runs): one instantiated graph of the op's
  // independent memcpy nodes per op (keyed by its word offset), launched as one submission
  std::map<size_t, hipGraphExec_t> batch_graphs_;
  void clear_batch_graphs();
  hipStream_t S(int64_t idx, hipStream_t main) const {
    // (graph capture keeps stream 0 on the capture's origin stream: a cycle of dependencies
    // among NON-origin streams crashes this runtime's hipStreamEndCapture, see side_stream_cycle)
    return idx == 0 ? (compute_ ? compute_ : (any_side_ && !graph_on_ ? home_ : main))
                    : streams_.at((size_t)idx);
  }
  int comm_cus_ = 0;
  // Stream-0 ops of a multi-stream plan run on `home_`, forked from and joined back into the
  // caller's stream; home_ and the side streams come from a process-wide pool (created once, in
  // a fixed order, never destroyed): the HIP stream -> hardware-queue mapping is fixed at
  // creation, and the one-GPU budget measured the SAME plan at 0.18 ms in one bind and 0.6-0.7
  // ms in the next when every bind created fresh streams beside the caller's null stream
  // (profiles/r04/r4_5_*). A single-stream plan stays on the caller's stream (no fork).
  hipStream_t home_ = nullptr;
  hipStream_t compute_ = nullptr;        // stream-0 ops under a CU split
  hipEvent_t compute_fork_ = nullptr, compute_join_ = nullptr;
  bool trace_on_ = false;
  std::vector<std::string> labels_;
  int device_;
  std::vector<hipStream_t> streams_;  // [0] unused (= caller stream)
  std::vector<hipEvent_t> events_;
  std::vector<hipEvent_t> fork_join_;  // one per stream
  std::vector<int64_t> ops_;
  std::vector<bool> used_;             // stream i touched by the plan
  // graph mode: before a cross-process wait (or a flag-gated GEMM) join the tails of every other
  // stream that already has ops, so ANY execution order of the captured graph keeps all ops
  // enqueued before the wait ahead of it (what makes the plan deadlock-free in one queue)
  std::vector<hipEvent_t> sync_ev_;
  std::vector<bool> touched_;  // graph capture: stream has an effectful op (not a wait / record)
  void join_others(int64_t stream, hipStream_t main);
  RcclComm* comm_ = nullptr;
  bool timeline_on_ = false;
  hipEvent_t tl_start_ = nullptr;
  std::vector<hipEvent_t> tl_ops_;
  std::vector<float> host_us_;
  unsigned epoch_ = 0;
  unsigned* d_timeout_ = nullptr;
  unsigned* d_epoch_ = nullptr;  // device copy of epoch_ (graph mode), inside d_timeout_'s block
};

}  // namespace ddlb
