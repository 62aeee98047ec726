// Plan executor implementation (see plan.h).
#include "plan.h"

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <chrono>
#include <functional>
#include <map>
#include <mutex>
#include <tuple>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "../gemm/gemm.h"
#include "kernels.h"

namespace ddlb {

namespace {

// roctx, resolved lazily from the library the Python side (ddlb_amd.utils.profiling) or the
// profiler already mapped, else loaded here: no link-time dependency on the tracer.
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
};
const Roctx& roctx() {
  static Roctx r = [] {
    Roctx x;
    const char* names[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                           "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", "libroctx64.so.4"};
    for (const char* n : names) {
      void* h = dlopen(n, RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
      if (!h) h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      x.push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
      x.pop = (int (*)())dlsym(h, "roctxRangePop");
      if (x.push && x.pop) break;
      x.push = nullptr;
      x.pop = nullptr;
    }
    return x;
  }();
  return r;
}

using BatchFn = hipError_t (*)(void**, void**, size_t*, size_t, hipMemcpyAttributes*, size_t*,
                               size_t, size_t*, hipStream_t);
BatchFn batch_fn() {
  static BatchFn f = [] {
    // look the symbol up in the HIP runtime this module is bound to (torch's copy)
    Dl_info info;
    BatchFn fn = nullptr;
    if (dladdr((void*)&hipMemcpyAsync, &info) && info.dli_fname) {
      void* h = dlopen(info.dli_fname, RTLD_NOW | RTLD_NOLOAD);
      if (h) fn = (BatchFn)dlsym(h, "hipMemcpyBatchAsync");
    }
    if (!fn) fn = (BatchFn)dlsym(RTLD_DEFAULT, "hipMemcpyBatchAsync");
    return fn;
  }();
  return f;
}

void crash_handler(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  static const char msg[] = "ddlb_amd: fatal signal, native backtrace follows\n";
  ssize_t w = write(2, msg, sizeof(msg) - 1);
  (void)w;
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

}  // namespace

bool copy_batch_api_available() { return batch_fn() != nullptr; }

namespace {
// what copy_batch actually did: a batch_memcpy timing is a batched-submission result
// only if the API call succeeded; otherwise it timed one hipMemcpyAsync per segment
int g_batch_state = 0;  // 0 not called, 1 batch API used, 2 fell back, 3 memcpy-node graph
std::string g_batch_error;
}  // namespace

std::string copy_batch_status() {
  if (g_batch_state == 3) return "hipGraph of memcpy nodes (one launch per batch)";
  if (batch_fn() == nullptr) return "unavailable (per-segment hipMemcpyAsync)";
  if (g_batch_state == 0) return "not called";
  if (g_batch_state == 1) return "hipMemcpyBatchAsync";
  return "fallback to per-segment hipMemcpyAsync: " + g_batch_error;
}

hipError_t copy_batch(void** dst, void** src, size_t* bytes, size_t n, hipStream_t s) {
  if (BatchFn fn = batch_fn(); fn && g_batch_state != 2) {
    size_t fail = 0;
    const hipError_t e = fn(dst, src, bytes, n, nullptr, nullptr, 0, &fail, s);
    if (e == hipSuccess) {
      g_batch_state = 1;
      return e;
    }
    (void)hipGetLastError();
    g_batch_state = 2;  // off after the first refusal (the header marks attrs unsupported)
    g_batch_error = hipGetErrorString(e);
  }
  if (batch_fn() == nullptr) g_batch_state = 2;
  for (size_t i = 0; i < n; ++i) {
    const hipError_t e = hipMemcpyAsync(dst[i], src[i], bytes[i], hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

void install_crash_handler() {
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_handler = crash_handler;
  sa.sa_flags = SA_RESETHAND;
  for (int sig : {SIGSEGV, SIGBUS, SIGABRT, SIGFPE}) sigaction(sig, &sa, nullptr);
}

namespace {
// Process-wide stream pool: slot s of priority class p on a device is created once (non-blocking)
// and reused by every executor (see PlanExecutor::home_). Slots are created in index order the
// first time an executor asks for them, so the home stream (slot 0) and the side streams of the
// first plan of a process land on consecutive hardware queues, and later plans get the same.
// cu_mask (optional, `words` 32-bit words): a CU-masked stream (hipExtStreamCreateWithCUMask);
// the mask is part of the key (a CU split's streams are pooled the same way).
hipStream_t pool_stream(int device, int slot, int prio_class, const uint32_t* cu_mask = nullptr,
                        int words = 0) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, std::vector<uint32_t>>, hipStream_t> pool;
  std::lock_guard<std::mutex> lock(mu);
  std::vector<uint32_t> mask(cu_mask, cu_mask + (cu_mask ? words : 0));
  auto key = std::make_tuple(device, slot, prio_class, mask);
  auto it = pool.find(key);
  if (it != pool.end()) return it->second;
  hipStream_t st = nullptr;
  if (cu_mask != nullptr) {
    DDLB_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)words, cu_mask));
  } else {
    int lo = 0, hi = 0;
    DDLB_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    DDLB_HIP(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, prio_class > 0 ? hi : lo));
  }
  pool[key] = st;
  return st;
}
}  // namespace

PlanExecutor::PlanExecutor(int device, int nstreams, int nevents,
                           const std::vector<int>& priorities)
    : device_(device) {
  DDLB_HIP(hipSetDevice(device));
  if (nstreams < 1) nstreams = 1;
  streams_.assign((size_t)nstreams, nullptr);
  fork_join_.assign((size_t)nstreams * 2, nullptr);
  used_.assign((size_t)nstreams, false);
  home_ = pool_stream(device, 0, 0);
  DDLB_HIP(hipEventCreateWithFlags(&compute_join_, hipEventDisableTiming));
  for (int i = 1; i < nstreams; ++i) {
    // priority: 0 = normal, 1 = high (comm streams)
    const int prio = (size_t)i < priorities.size() ? priorities[(size_t)i] : 0;
    streams_[(size_t)i] = pool_stream(device, i, prio > 0 ? 1 : 0);
  }
  for (auto& e : fork_join_) DDLB_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  sync_ev_.assign((size_t)nstreams, nullptr);
  for (auto& e : sync_ev_) DDLB_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  touched_.assign((size_t)nstreams, false);
  events_.assign((size_t)(nevents > 0 ? nevents : 0), nullptr);
  for (auto& e : events_) DDLB_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  DDLB_HIP(hipMalloc(&d_timeout_, 256));
  DDLB_HIP(hipMemset(d_timeout_, 0, 256));
  d_epoch_ = d_timeout_ + 32;  // its own 128-byte line of the same allocation
}

void PlanExecutor::clear_batch_graphs() {
  for (auto& kv : batch_graphs_)
    if (kv.second) hipGraphExecDestroy(kv.second);
  batch_graphs_.clear();
}

PlanExecutor::~PlanExecutor() {
  hipSetDevice(device_);
  clear_batch_graphs();
  if (tl_start_) hipEventDestroy(tl_start_);
  for (auto e : tl_ops_) if (e) hipEventDestroy(e);
  if (graph_exec_) hipGraphExecDestroy(graph_exec_);
  if (graph_) hipGraphDestroy(graph_);
  if (cap_stream_) hipStreamDestroy(cap_stream_);
  if (compute_) hipStreamSynchronize(compute_);  // a pool stream
  if (compute_fork_) hipEventDestroy(compute_fork_);
  if (compute_join_) hipEventDestroy(compute_join_);
  if (home_) hipStreamSynchronize(home_);
  for (size_t i = 1; i < streams_.size(); ++i)
    if (streams_[i]) hipStreamSynchronize(streams_[i]);  // pool streams live on
  for (auto e : fork_join_) if (e) hipEventDestroy(e);
  for (auto e : sync_ev_) if (e) hipEventDestroy(e);
  for (auto e : events_) if (e) hipEventDestroy(e);
  if (d_timeout_) hipFree(d_timeout_);
}

void PlanExecutor::load(const std::vector<int64_t>& ops) {
  validate_ops(ops, streams_.size(), events_.size());  // plan_ir.h: every bound exec relies on
  used_ = used_streams(ops, streams_.size());
  ops_ = ops;
  clear_batch_graphs();
  if (timeline_on_) set_timeline(true);  // one timing event per (new) op
  any_side_ = false;
  for (size_t i = 1; i < used_.size(); ++i) any_side_ = any_side_ || used_[i];
  if (graph_exec_) { hipGraphExecDestroy(graph_exec_); graph_exec_ = nullptr; }
  if (graph_) { hipGraphDestroy(graph_); graph_ = nullptr; }
}

bool PlanExecutor::graph_capturable() const {
  // In graph mode the epoch-dependent ops (cross-process signals / waits, the in-kernel
  // all-gather's flags) read the run counter from device memory (d_epoch_, bumped by the first
  // node of every replay) instead of a value baked in at enqueue time, so they capture. Not
  // captured:
  //  * RCCL calls: replaying a captured RCCL collective crashed the process on this image
  //    (torch's RCCL 2.26, profiles/r02/r2_19*); RCCL plans issue few calls per run anyway.
  //  * a flag-gated GEMM whose flags other streams set (the fused copy-engine pipelines): the
  //    graph may place it ahead of the copy / signal nodes in one hardware queue, and its
  //    spinning tiles would then wait for nodes queued behind them; ordering it after every
  //    copy stream instead serialises copy-then-GEMM and removes the overlap it exists for
  //    (ADVICE r2). Such plans run eagerly, where the enqueue order puts the copies first.
  //  * a CU split (set_cu_split): masked streams are not carried into graph nodes.
  //  * a cycle of dependencies among the side streams (s -> t and, later, t -> s, through event
  //    edges or the joins before cross-process waits; no cycle of nodes needed):
  //    hipStreamEndCapture of this HIP runtime segfaults on it (scripts/diag_graph_edges.py
  //    `cycle`, profiles/r03/r3_15_*). Cycles through the capture's origin stream (the fork /
  //    join every plan has) are fine.
  if (comm_cus_ > 0 || has_uncapturable_op(ops_)) return false;
  return !side_stream_cycle(ops_, streams_.size(), events_.size());
}

void PlanExecutor::enable_graph(bool on) {
  if (on && timeline_on_) throw std::runtime_error("hipGraph replay: turn the plan timeline off");
  if (on && !graph_capturable())
    throw std::runtime_error("hipGraph replay: plans with RCCL calls, copy-engine-fed "
                             "flag-gated GEMMs, a CU split or a cycle among side streams are not "
                             "captured (see PlanExecutor::graph_capturable)");
  if (on) {  // the device run counter continues from the host one (see graph_capturable)
    DDLB_HIP(hipSetDevice(device_));
    DDLB_HIP(hipDeviceSynchronize());
    DDLB_HIP(hipMemcpy(d_epoch_, &epoch_, sizeof(unsigned), hipMemcpyHostToDevice));
  }
  graph_on_ = on;
  if (on && cap_stream_ == nullptr) {
    DDLB_HIP(hipStreamCreateWithFlags(&cap_stream_, hipStreamNonBlocking));
  }
}

void PlanExecutor::set_cu_split(int comm_cus) {
  if (comm_cus == comm_cus_) return;
  if (graph_on_) throw std::runtime_error("CU split: not with hipGraph replay");
  if (comm_cus_ != 0) throw std::runtime_error("CU split: set once per executor");
  DDLB_HIP(hipSetDevice(device_));
  int ncu = 0;
  DDLB_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device_));
  if (comm_cus < 0 || comm_cus >= ncu)
    throw std::runtime_error("CU split: comm_cus must be in [0, " + std::to_string(ncu) + ")");
  DDLB_HIP(hipDeviceSynchronize());
  // mask bit i = CU i (the driver spreads consecutive bits over the XCDs / shader engines)
  const int words = (ncu + 31) / 32;
  std::vector<uint32_t> comm((size_t)words, 0u), comp((size_t)words, 0u);
  for (int i = 0; i < ncu; ++i) (i < comm_cus ? comm : comp)[(size_t)(i / 32)] |= 1u << (i % 32);
  // masked streams come from the pool too (keyed by their mask): see home_ in plan.h
  compute_ = pool_stream(device_, 0, 0, comp.data(), words);
  for (size_t i = 1; i < streams_.size(); ++i)
    streams_[i] = pool_stream(device_, (int)i, 0, comm.data(), words);
  DDLB_HIP(hipEventCreateWithFlags(&compute_fork_, hipEventDisableTiming));
  comm_cus_ = comm_cus;
}

std::vector<std::vector<int>> PlanExecutor::stream_info() const {
  std::vector<std::vector<int>> out;
  auto one = [&](int idx, hipStream_t st) {
    unsigned flags = 0;
    int prio = 0;
    DDLB_HIP(hipStreamGetFlags(st, &flags));
    DDLB_HIP(hipStreamGetPriority(st, &prio));
    out.push_back({idx, (int)flags, prio});
  };
  for (size_t i = 1; i < streams_.size(); ++i)
    if (streams_[i]) one((int)i, streams_[i]);
  if (compute_) one(-1, compute_);
  return out;
}

void PlanExecutor::set_trace(bool on, const std::vector<std::string>& labels) {
  if (on && (roctx().push == nullptr))
    throw std::runtime_error("plan trace: no roctx library (librocprofiler-sdk-roctx) found");
  trace_on_ = on;
  labels_ = labels;
}

unsigned PlanExecutor::read_timeout() {
  unsigned v = 0;
  DDLB_HIP(hipMemcpy(&v, d_timeout_, sizeof(v), hipMemcpyDeviceToHost));
  return v;
}

void PlanExecutor::set_timeline(bool on) {
  if (on && graph_on_) throw std::runtime_error("plan timeline: not available with hipGraph replay");
  DDLB_HIP(hipSetDevice(device_));
  if (on && tl_start_ == nullptr) DDLB_HIP(hipEventCreate(&tl_start_));
  const size_t n = ops_.size() / kOpWords;
  while (on && tl_ops_.size() < n) {
    hipEvent_t e = nullptr;
    DDLB_HIP(hipEventCreate(&e));
    tl_ops_.push_back(e);
  }
  timeline_on_ = on;
}

std::vector<float> PlanExecutor::timeline() {
  if (!timeline_on_) throw std::runtime_error("plan timeline: call set_timeline(true) and run()");
  const size_t n = ops_.size() / kOpWords;
  std::vector<float> out(n, 0.f);
  for (size_t i = 0; i < n; ++i) {
    DDLB_HIP(hipEventSynchronize(tl_ops_[i]));
    DDLB_HIP(hipEventElapsedTime(&out[i], tl_start_, tl_ops_[i]));
  }
  return out;
}

// DDLB_GRAPH_DEBUG=1: a stderr line per capture / instantiate / launch step and per captured op
// (op code, stream, graph node count), flushed, to locate a crash inside the runtime.
static bool graph_debug() {
  static const bool on = getenv("DDLB_GRAPH_DEBUG") != nullptr;
  return on;
}
#define GDBG(...)                                  \
  do {                                             \
    if (graph_debug()) {                           \
      fprintf(stderr, "[graph] " __VA_ARGS__);     \
      fputc('\n', stderr);                         \
      fflush(stderr);                              \
    }                                              \
  } while (0)

void PlanExecutor::join_others(int64_t stream, hipStream_t main) {
  hipStream_t s = S(stream, main);
  for (size_t j = 0; j < streams_.size(); ++j) {
    if ((int64_t)j == stream || !touched_[j]) continue;
    DDLB_HIP(hipEventRecord(sync_ev_[j], S((int64_t)j, main)));
    DDLB_HIP(hipStreamWaitEvent(s, sync_ev_[j], 0));
  }
}

void PlanExecutor::enqueue(hipStream_t main) {
  std::fill(touched_.begin(), touched_.end(), false);
  if (timeline_on_) DDLB_HIP(hipEventRecord(tl_start_, main));
  size_t first = 0;
  if (graph_on_) {
    // first node of every replay: the run-counter bump, fused with the plan's leading signals on
    // the main stream (READY to the peers, own-shard arrival flags): one launch instead of 1 + k
    // (each small kernel after a GEMM costs a few us of boundary + L2 write-back)
    BumpSignalArgs b;
    b.epoch = d_epoch_;
    first = fused_prologue(ops_, b);
    if (first > 0) touched_[0] = true;
    DDLB_HIP(bump_signal_launch(b, main));
  }
  if (any_side_ || compute_) {
    // fork: every used side stream and the stream-0 stream (home, or the CU-split compute
    // stream) wait for everything already queued on `main`
    DDLB_HIP(hipEventRecord(fork_join_[0], main));
    for (size_t i = 1; i < streams_.size(); ++i)
      if (used_[i]) DDLB_HIP(hipStreamWaitEvent(streams_[i], fork_join_[0], 0));
    if (S(0, main) != main) DDLB_HIP(hipStreamWaitEvent(S(0, main), fork_join_[0], 0));
  }
  if (timeline_on_) host_us_.assign(ops_.size() / kOpWords, 0.f);
  for (size_t i = first; i < ops_.size(); i += kOpWords) {
    const int64_t* o = &ops_[i];
    // graph mode: a cross-process wait is ordered after everything enqueued before it on any
    // stream (the deadlock-freedom argument of the eager enqueue order, kept under any node
    // order the graph may pick); flag-gated GEMMs fed by other streams are not captured at all
    if (graph_on_ && o[0] == OP_WAIT_SIGNAL) join_others(o[1], main);
    // only ops with an effect a peer can depend on count: waits and event records add none, and
    // joining a wait-only stream would create side-stream -> side-stream capture relations that,
    // together with the plan's own side-stream edges (copy_streams > 1), form a cycle on which
    // this HIP runtime's hipStreamEndCapture segfaults (scripts/diag_graph_edges.py cs2_exact)
    if (o[0] != OP_WAIT_SIGNAL && o[0] != OP_WAIT && o[0] != OP_RECORD) touched_[(size_t)o[1]] = true;
    const size_t idx = i / kOpWords;
    if (graph_on_) GDBG("  op %zu code %lld stream %lld", idx, (long long)o[0], (long long)o[1]);
    const bool tr = trace_on_ && idx < labels_.size();
    if (tr) roctx().push(labels_[idx].c_str());
    if (!timeline_on_) {
      exec(&ops_[i], main);
      if (graph_on_) GDBG("  op %zu enqueued", idx);
      if (tr) roctx().pop();
      continue;
    }
    const auto t0 = std::chrono::steady_clock::now();
    exec(&ops_[i], main);
    const auto t1 = std::chrono::steady_clock::now();
    host_us_[idx] = std::chrono::duration<float, std::micro>(t1 - t0).count();
    DDLB_HIP(hipEventRecord(tl_ops_[idx], S(ops_[i + 1], main)));
    if (tr) roctx().pop();
  }
  if (any_side_) {  // join
    for (size_t i = 1; i < streams_.size(); ++i)
      if (used_[i]) {
        if (graph_on_) GDBG("  join stream %zu", i);
        DDLB_HIP(hipEventRecord(fork_join_[streams_.size() + i], streams_[i]));
        DDLB_HIP(hipStreamWaitEvent(main, fork_join_[streams_.size() + i], 0));
      }
  }
  if (graph_on_) GDBG("  enqueue done");
  if (S(0, main) != main) {
    DDLB_HIP(hipEventRecord(compute_join_, S(0, main)));
    DDLB_HIP(hipStreamWaitEvent(main, compute_join_, 0));
  }
}

unsigned PlanExecutor::run(uintptr_t main_stream) {
  hipStream_t main = (hipStream_t)main_stream;
  ++epoch_;
  if (!graph_on_) {
    enqueue(main);
    return epoch_;
  }
  if (graph_exec_ == nullptr) {
    // capture on a private stream (the caller's may be the legacy null stream)
    GDBG("begin capture (%zu ops, %zu streams)", ops_.size() / kOpWords, streams_.size());
    DDLB_HIP(hipStreamBeginCapture(cap_stream_, hipStreamCaptureModeRelaxed));
    try {
      enqueue(cap_stream_);
    } catch (...) {
      hipGraph_t g = nullptr;
      hipStreamEndCapture(cap_stream_, &g);
      if (g) hipGraphDestroy(g);
      throw;
    }
    DDLB_HIP(hipStreamEndCapture(cap_stream_, &graph_));
    if (graph_debug()) {
      size_t nn = 0;
      hipGraphGetNodes(graph_, nullptr, &nn);
      std::vector<hipGraphNode_t> nodes(nn);
      hipGraphGetNodes(graph_, nodes.data(), &nn);
      int counts[16] = {0};
      for (auto n : nodes) {
        hipGraphNodeType t;
        if (hipGraphNodeGetType(n, &t) == hipSuccess && (int)t >= 0 && (int)t < 16) ++counts[(int)t];
      }
      GDBG("end capture: %zu nodes (kernel %d memcpy %d memset %d host %d graph %d empty %d "
           "wait_event %d event_record %d)", nn, counts[hipGraphNodeTypeKernel],
           counts[hipGraphNodeTypeMemcpy], counts[hipGraphNodeTypeMemset],
           counts[hipGraphNodeTypeHost], counts[hipGraphNodeTypeGraph],
           counts[hipGraphNodeTypeEmpty], counts[hipGraphNodeTypeWaitEvent],
           counts[hipGraphNodeTypeEventRecord]);
    }
    DDLB_HIP(hipGraphInstantiate(&graph_exec_, graph_, nullptr, nullptr, 0));
    GDBG("instantiated");
  }
  GDBG("launch epoch %u", epoch_);
  DDLB_HIP(hipGraphLaunch(graph_exec_, main));
  GDBG("launched");
  if (graph_debug()) {
    DDLB_HIP(hipStreamSynchronize(main));
    GDBG("synchronized");
  }
  return epoch_;
}

GemmArgs PlanExecutor::gemm_args(const int64_t* o) const {
  GemmArgs g = decode_gemm(o);  // plan_ir.h
  g.epoch = epoch_;
  g.timeout_word = d_timeout_;
  // DDLB_SPIN_LIMIT: polls before a gated GEMM's bounded spin gives up (diagnostics that provoke
  // a blocked producer on purpose, research/diag/diag_gate_placement.py); default ~30 s
  static const unsigned spin_env = getenv("DDLB_SPIN_LIMIT") ? (unsigned)atol(getenv("DDLB_SPIN_LIMIT")) : 0u;
  if (spin_env > 0) g.spin_limit = spin_env;
  g.epoch_ptr = graph_on_ ? d_epoch_ : nullptr;
  return g;
}

void PlanExecutor::exec(const int64_t* o, hipStream_t main) {
  hipStream_t s = S(o[1], main);
  switch (o[0]) {
    case OP_NOP: return;
    case OP_GEMM: {
      const GemmArgs g = gemm_args(o);
      DDLB_HIP(gemm_launch(g, (int)o[15], (int)o[16], (int)o[17], (int)o[18], s));
      return;
    }
    case OP_RECORD: DDLB_HIP(hipEventRecord(events_[(size_t)o[2]], s)); return;
    case OP_WAIT: DDLB_HIP(hipStreamWaitEvent(s, events_[(size_t)o[2]], 0)); return;
    case OP_ALLGATHER:
      if (!comm_) throw std::runtime_error("plan: allgather without an RCCL communicator");
      DDLB_NCCL(ncclAllGather((const void*)o[2], (void*)o[3], (size_t)o[4], nccl_dtype((int)o[5]),
                              comm_->get(), s));
      return;
    case OP_REDUCE_SCATTER:
      if (!comm_) throw std::runtime_error("plan: reduce-scatter without an RCCL communicator");
      DDLB_NCCL(ncclReduceScatter((const void*)o[2], (void*)o[3], (size_t)o[4],
                                  nccl_dtype((int)o[5]), ncclSum, comm_->get(), s));
      return;
    case OP_SEND:
      if (!comm_) throw std::runtime_error("plan: send without an RCCL communicator");
      DDLB_NCCL(ncclSend((const void*)o[2], (size_t)o[3], nccl_dtype((int)o[4]), (int)o[5],
                         comm_->get(), s));
      return;
    case OP_RECV:
      if (!comm_) throw std::runtime_error("plan: recv without an RCCL communicator");
      DDLB_NCCL(ncclRecv((void*)o[2], (size_t)o[3], nccl_dtype((int)o[4]), (int)o[5],
                         comm_->get(), s));
      return;
    case OP_GROUP_START: DDLB_NCCL(ncclGroupStart()); return;
    case OP_GROUP_END: DDLB_NCCL(ncclGroupEnd()); return;
    case OP_COPY:
      if (o[5] == 0) {
        DDLB_HIP(hipMemcpyAsync((void*)o[2], (const void*)o[3], (size_t)o[4],
                                hipMemcpyDeviceToDevice, s));
      } else {
        CopyArgs c;
        c.nseg = 1;
        c.dst[0] = (void*)o[2];
        c.src[0] = (const void*)o[3];
        c.bytes[0] = o[4];
        DDLB_HIP(copy_launch(c, (int)o[6], s));
      }
      return;
    case OP_COPY_BATCH: {
      const int n = (int)o[2];
      if (n < 1 || n > kMaxCopySeg || 4 + 3 * n > kOpWords)
        throw std::runtime_error("plan: bad batch copy");
      void* dst[kMaxCopySeg];
      void* src[kMaxCopySeg];
      size_t bytes[kMaxCopySeg];
      for (int i = 0; i < n; ++i) {
        dst[i] = (void*)o[4 + 3 * i];
        src[i] = (void*)o[5 + 3 * i];
        bytes[i] = (size_t)o[6 + 3 * i];
      }
      if (graph_on_) {  // captured as memcpy nodes (the batch API is not a capturable call)
        for (int i = 0; i < n; ++i)
          DDLB_HIP(hipMemcpyAsync(dst[i], src[i], bytes[i], hipMemcpyDeviceToDevice, s));
      } else if (copy_batch_api_available()) {
        DDLB_HIP(copy_batch(dst, src, bytes, (size_t)n, s));
      } else {
        // no batch API in this HIP runtime: the op's segments as ONE submission anyway, a graph
        // of n independent memcpy nodes (instantiated once per op; the addresses are fixed at
        // bind), so the engines take every peer's segment at once instead of n serial copies
        const size_t key = (size_t)(o - ops_.data());
        auto it = batch_graphs_.find(key);
        if (it == batch_graphs_.end()) {
          hipGraph_t g = nullptr;
          DDLB_HIP(hipGraphCreate(&g, 0));
          for (int i = 0; i < n; ++i) {
            hipGraphNode_t node;
            DDLB_HIP(hipGraphAddMemcpyNode1D(&node, g, nullptr, 0, dst[i], src[i], bytes[i],
                                             hipMemcpyDeviceToDevice));
          }
          hipGraphExec_t ex = nullptr;
          const hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
          hipGraphDestroy(g);
          DDLB_HIP(e);
          it = batch_graphs_.emplace(key, ex).first;
        }
        DDLB_HIP(hipGraphLaunch(it->second, s));
        g_batch_state = 3;
      }
      return;
    }
    case OP_COPY_MULTI: {
      CopyArgs c;
      c.nseg = (int)o[2];
      if (c.nseg < 1 || c.nseg > kMaxCopySeg || 4 + 3 * c.nseg > kOpWords)
        throw std::runtime_error("plan: bad multi-copy");
      for (int i = 0; i < c.nseg; ++i) {
        c.dst[i] = (void*)o[4 + 3 * i];
        c.src[i] = (const void*)o[5 + 3 * i];
        c.bytes[i] = o[6 + 3 * i];
      }
      DDLB_HIP(copy_launch(c, (int)o[3], s));
      return;
    }
    case OP_SIGNAL: {
      const int n = (int)o[2];
      if (n < 1 || n > kMaxSignal || 5 + n > kOpWords) throw std::runtime_error("plan: bad signal");
      const unsigned value = (unsigned)((int64_t)epoch_ + o[4]);
      if (o[3] == 1 && !graph_on_) {
        for (int i = 0; i < n; ++i) DDLB_HIP(hipStreamWriteValue32(s, (void*)o[5 + i], value, 0));
      } else {
        SignalArgs a;  // graph mode: always the kernel, reading the device run counter
        a.n = n;
        a.value = value;
        if (graph_on_) {
          a.epoch_ptr = d_epoch_;
          a.delta = (int)o[4];
        }
        for (int i = 0; i < n; ++i) a.ptr[i] = (unsigned*)o[5 + i];
        DDLB_HIP(signal_launch(a, s));
      }
      return;
    }
    case OP_WAIT_SIGNAL: {
      const int n = (int)o[2];
      if (n < 1 || n > kMaxSignal || 5 + n > kOpWords) throw std::runtime_error("plan: bad wait");
      if (o[3] == 2) return;  // performed inside the preceding in-kernel all-gather launch
      const int64_t v = (int64_t)epoch_ + o[4];
      if (v <= 0 && !graph_on_) return;  // nothing to wait for before the first epoch
      if (o[3] == 1 && !graph_on_) {
        for (int i = 0; i < n; ++i)
          DDLB_HIP(hipStreamWaitValue32(s, (void*)o[5 + i], (unsigned)v, hipStreamWaitValueGte,
                                        0xffffffffu));
      } else {
        WaitArgs a;
        a.n = n;
        a.value = v > 0 ? (unsigned)v : 0u;
        a.timeout_word = d_timeout_;
        if (graph_on_) {
          a.epoch_ptr = d_epoch_;
          a.delta = (int)o[4];
        }
        for (int i = 0; i < n; ++i) a.ptr[i] = (unsigned*)o[5 + i];
        DDLB_HIP(wait_launch(a, s));
      }
      return;
    }
    case OP_REDUCE: {
      ReduceArgs a;
      a.dst = (void*)o[2];
      a.count = o[3];
      a.nsrc = (int)o[5];
      if (a.nsrc < 1 || a.nsrc > kMaxReduceSrc || 6 + a.nsrc > kOpWords)
        throw std::runtime_error("plan: bad reduce");
      for (int i = 0; i < a.nsrc; ++i) a.src[i] = (const void*)o[6 + i];
      const int dt = (int)o[4];
      const int kdt = dt == DT_F32 ? 0 : dt == DT_F16 ? 1 : dt == DT_BF16 ? 2 : -1;
      if (kdt < 0) throw std::runtime_error("plan: reduce dtype must be f32/f16/bf16");
      DDLB_HIP(reduce_sum_launch(a, kdt, s));
      return;
    }
    case OP_MEMSET:
      DDLB_HIP(hipMemsetAsync((void*)o[2], (int)o[4], (size_t)o[3], s));
      return;
    default:
      throw std::runtime_error("plan: unknown op kind " + std::to_string(o[0]));
  }
}

}  // namespace ddlb
