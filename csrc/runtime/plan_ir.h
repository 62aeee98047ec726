// Plan IR: the host-only half of the plan executor (csrc/runtime/plan.cpp) -- op-word decoding,
// validation and the stream / event bookkeeping that decides graph capture. No HIP call lives
// here, so tests/native/test_plan_ir.cpp builds it for the host alone under AddressSanitizer +
// UndefinedBehaviorSanitizer and feeds it every plan the simulator tests build (SURVEY.md §5.2:
// sanitizer builds of the C++ layer; the GPU side has no sanitizer on this pool).
//
// Layout (kOpWords int64 per op; word 0 = kind, word 1 = stream index) and the op kinds are in
// plan.h; the Python encoder is ddlb_amd/parallel/plan.py Plan.encode.
#pragma once
#include <stdint.h>

#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../gemm/gemm.h"
#include "kernels.h"

namespace ddlb {

constexpr int kOpWords = 34;
enum OpKind : int64_t {
  OP_NOP = 0,
  OP_GEMM = 1,        // 2 a, 3 b, 4 c, 5 lda, 6 ldb, 7 ldc, 8 a_grp, 9 a_gstride, 10 c_grp,
                      // 11 c_gstride, 12 M, 13 N, 14 K, 15 din, 16 dout, 17 tile, 18 mode,
                      // 19 flags ptr (0 = none), 20 flag_rows, 21 nshards, 22 first_shard,
                      // 23 tile_order, 24 fused epilogue activation, 25 A shard table,
                      // 26 A shard rows, 27 nsub, 28 reserve_cus, 29 in-kernel all-gather
                      // (ctas | parts << 20 | rank << 40 | mode << 56), 30 its table,
                      // 31 K-split slices, 32 C shard table (direct store), 33 C shard rows
  OP_RECORD = 2,      // 2 event
  OP_WAIT = 3,        // 2 event
  OP_ALLGATHER = 4,   // 2 send, 3 recv, 4 count per rank, 5 dtype
  OP_REDUCE_SCATTER = 5,  // 2 send, 3 recv, 4 recv count, 5 dtype
  OP_SEND = 6,        // 2 buf, 3 count, 4 dtype, 5 peer
  OP_RECV = 7,        // 2 buf, 3 count, 4 dtype, 5 peer
  OP_GROUP_START = 8,
  OP_GROUP_END = 9,
  OP_COPY = 10,       // 2 dst, 3 src, 4 bytes, 5 method (0 copy engine, 1 CU kernel),
                      // 6 max CU blocks (kernel method)
  OP_SIGNAL = 11,     // 2 n, 3 method (0 kernel, 1 stream write), 4 delta, 5.. flag ptrs;
                      //   stores value = epoch + delta
  OP_WAIT_SIGNAL = 12,  // 2 n, 3 method (0 kernel, 1 stream wait, 2 inside the preceding
                        //   in-kernel all-gather), 4 delta, 5.. flag ptrs; waits until every
                        //   flag >= epoch + delta
  OP_REDUCE = 13,     // 2 dst, 3 count, 4 dtype, 5 nsrc, 6.. src ptrs
  OP_MEMSET = 14,     // 2 dst, 3 bytes, 4 byte value
  OP_COPY_MULTI = 15, // 2 nseg, 3 max blocks, then (dst, src, bytes) triples from word 4
  OP_COPY_BATCH = 16, // 2 nseg, then (dst, src, bytes) triples from word 4: copy-engine copies
                      //   submitted as ONE hipMemcpyBatchAsync (multicast_protocol=batch_memcpy)
};
constexpr int64_t kLastOpKind = OP_COPY_BATCH;

[[noreturn]] inline void plan_error(size_t op, const std::string& what) {
  throw std::runtime_error("plan op " + std::to_string(op) + ": " + what);
}

// Every check the executor relies on, at load time (so a bad plan is refused before anything is
// enqueued): array length, stream / event indices, each kind's counts against the op size and
// the kernels' argument arrays, non-null operands, non-negative sizes.
inline void validate_ops(const std::vector<int64_t>& ops, size_t nstreams, size_t nevents) {
  if (ops.size() % kOpWords != 0) throw std::runtime_error("plan: bad op array length");
  for (size_t i = 0, idx = 0; i < ops.size(); i += kOpWords, ++idx) {
    const int64_t* o = &ops[i];
    if (o[0] < OP_NOP || o[0] > kLastOpKind) plan_error(idx, "unknown op kind " + std::to_string(o[0]));
    if (o[1] < 0 || (size_t)o[1] >= nstreams) plan_error(idx, "bad stream index");
    switch (o[0]) {
      case OP_RECORD: case OP_WAIT:
        if (o[2] < 0 || (size_t)o[2] >= nevents) plan_error(idx, "bad event index");
        break;
      case OP_GEMM:
        if (o[12] < 0 || o[13] < 0 || o[14] <= 0) plan_error(idx, "bad GEMM shape");
        if (o[12] >= (int64_t)1 << 31 || o[13] >= (int64_t)1 << 31 || o[14] >= (int64_t)1 << 31)
          plan_error(idx, "GEMM dimension beyond 32 bits");
        if (!o[2] || !o[3] || !o[4]) plan_error(idx, "null GEMM ptr");
        if (o[5] < 0 || o[6] < 0 || o[7] < 0) plan_error(idx, "negative GEMM leading dimension");
        if (o[31] < 0 || o[31] > 64) plan_error(idx, "bad K-split");
        if (o[29] != 0 && (o[19] == 0 || o[30] == 0)) plan_error(idx, "all-gather without flags / table");
        break;
      case OP_ALLGATHER: case OP_REDUCE_SCATTER:
        if (!o[2] || !o[3] || o[4] < 0) plan_error(idx, "bad collective");
        break;
      case OP_SEND: case OP_RECV:
        if (!o[2] || o[3] < 0 || o[5] < 0) plan_error(idx, "bad send / recv");
        break;
      case OP_COPY:
        if (!o[2] || !o[3] || o[4] < 0 || (o[5] != 0 && o[5] != 1)) plan_error(idx, "bad copy");
        break;
      case OP_COPY_BATCH: case OP_COPY_MULTI: {
        const int64_t n = o[2];
        if (n < 1 || n > kMaxCopySeg || 4 + 3 * n > kOpWords) plan_error(idx, "bad multi-segment copy");
        for (int64_t j = 0; j < n; ++j)
          if (!o[4 + 3 * j] || !o[5 + 3 * j] || o[6 + 3 * j] < 0) plan_error(idx, "bad copy segment");
        break;
      }
      case OP_SIGNAL: case OP_WAIT_SIGNAL: {
        const int64_t n = o[2];
        if (n < 1 || n > kMaxSignal || 5 + n > kOpWords) plan_error(idx, "bad signal count");
        if (o[3] < 0 || o[3] > (o[0] == OP_SIGNAL ? 1 : 2)) plan_error(idx, "bad signal method");
        for (int64_t j = 0; j < n; ++j)
          if (!o[5 + j]) plan_error(idx, "null flag");
        break;
      }
      case OP_REDUCE: {
        const int64_t n = o[5];
        if (n < 1 || n > kMaxReduceSrc || 6 + n > kOpWords) plan_error(idx, "bad reduce");
        if (o[4] != DT_F32 && o[4] != DT_F16 && o[4] != DT_BF16)
          plan_error(idx, "reduce dtype must be f32/f16/bf16");
        if (!o[2] || o[3] < 0) plan_error(idx, "bad reduce destination");
        for (int64_t j = 0; j < n; ++j)
          if (!o[6 + j]) plan_error(idx, "null reduce source");
        break;
      }
      case OP_MEMSET:
        if (!o[2] || o[3] < 0) plan_error(idx, "bad memset");
        break;
      default: break;
    }
  }
}

// Streams the plan uses ([0] = the caller's stream).
inline std::vector<bool> used_streams(const std::vector<int64_t>& ops, size_t nstreams) {
  std::vector<bool> used(nstreams, false);
  for (size_t i = 0; i < ops.size(); i += kOpWords)
    if (ops[i + 1] >= 0 && (size_t)ops[i + 1] < nstreams) used[(size_t)ops[i + 1]] = true;
  return used;
}

// GemmArgs of an OP_GEMM, as far as the op words define it (the executor adds the run's epoch,
// its device words and the spin bound).
inline GemmArgs decode_gemm(const int64_t* o) {
  GemmArgs g;
  g.a = (const void*)o[2];
  g.b = (const void*)o[3];
  g.c = (void*)o[4];
  g.lda = o[5]; g.ldb = o[6]; g.ldc = o[7];
  g.a_grp = o[8]; g.a_gstride = o[9];
  g.c_grp = o[10]; g.c_gstride = o[11];
  g.M = (int)o[12]; g.N = (int)o[13]; g.K = (int)o[14];
  g.flags = (const unsigned*)o[19];
  g.flag_rows = o[20] > 0 ? o[20] : 1;
  g.nshards = o[21] > 0 ? (int)o[21] : 1;
  g.first_shard = (int)o[22];
  g.tile_order = (int)o[23];
  g.act = (int)o[24];
  g.a_table = (const uint64_t*)o[25];
  g.shard_rows = o[26];
  g.nsub = o[27] > 0 ? (int)o[27] : 1;
  g.reserve_cus = (int)o[28];
  g.ag_ctas = (int)(o[29] & 0xfffff);
  g.ag_parts = (int)((o[29] >> 20) & 0xfffff);
  g.ag_rank = (int)((o[29] >> 40) & 0xffff);
  g.ag_mode = (int)((o[29] >> 56) & 0x7f);
  g.ag_tab = (const uint64_t*)o[30];
  g.ksplit = o[31] > 1 ? (int)o[31] : 1;
  g.c_table = (const uint64_t*)o[32];
  g.c_shard_rows = o[33];
  return g;
}

// Ops whose capture this runtime cannot replay (see PlanExecutor::graph_capturable): RCCL calls,
// and a flag-gated GEMM fed by other streams (not by its own in-kernel all-gather).
inline bool has_uncapturable_op(const std::vector<int64_t>& ops) {
  for (size_t i = 0; i < ops.size(); i += kOpWords) {
    const int64_t k = ops[i];
    if (k == OP_ALLGATHER || k == OP_REDUCE_SCATTER || k == OP_SEND || k == OP_RECV ||
        k == OP_GROUP_START || k == OP_GROUP_END)
      return true;
    if (k == OP_GEMM && ops[i + 19] != 0 && ops[i + 29] == 0) return true;
  }
  return false;
}

// A cycle of dependencies among the side streams (stream 0 excluded) as a graph-mode enqueue
// creates them: event edges (record on s, wait on t) and the joins before every cross-process
// wait (every stream with an effectful op so far -> the waiting stream).
inline bool side_stream_cycle(const std::vector<int64_t>& ops, size_t nstreams, size_t nevents) {
  const size_t ns = nstreams;
  std::vector<std::vector<char>> adj(ns, std::vector<char>(ns, 0));
  std::vector<int64_t> rec_on(nevents, -1);
  std::vector<char> effect(ns, 0);
  auto edge = [&](int64_t a, int64_t b) {
    if (a >= 1 && b >= 1 && a != b && (size_t)a < ns && (size_t)b < ns) adj[(size_t)a][(size_t)b] = 1;
  };
  for (size_t i = 0; i < ops.size(); i += kOpWords) {
    const int64_t k = ops[i], st = ops[i + 1];
    if (k == OP_RECORD && ops[i + 2] >= 0 && (size_t)ops[i + 2] < rec_on.size())
      rec_on[(size_t)ops[i + 2]] = st;
    if (k == OP_WAIT && ops[i + 2] >= 0 && (size_t)ops[i + 2] < rec_on.size())
      edge(rec_on[(size_t)ops[i + 2]], st);
    if (k == OP_WAIT_SIGNAL)
      for (size_t j = 0; j < ns; ++j)
        if (effect[j]) edge((int64_t)j, st);
    if (k != OP_WAIT_SIGNAL && k != OP_WAIT && k != OP_RECORD && st >= 0 && (size_t)st < ns)
      effect[(size_t)st] = 1;
  }
  std::vector<int> colour(ns, 0);  // colour DFS over at most a few dozen streams
  std::function<bool(size_t)> dfs = [&](size_t u) {
    colour[u] = 1;
    for (size_t v = 0; v < ns; ++v) {
      if (!adj[u][v]) continue;
      if (colour[v] == 1 || (colour[v] == 0 && dfs(v))) return true;
    }
    colour[u] = 2;
    return false;
  };
  for (size_t u = 1; u < ns; ++u)
    if (colour[u] == 0 && dfs(u)) return true;
  return false;
}

// The leading stream-0 signals a graph replay fuses into its first node (the run-counter bump):
// the number of op words they span, and their (flag, delta) pairs appended to `b`.
inline size_t fused_prologue(const std::vector<int64_t>& ops, BumpSignalArgs& b) {
  size_t first = 0;
  for (; first < ops.size(); first += kOpWords) {
    const int64_t* o = &ops[first];
    if (o[0] != OP_SIGNAL || o[1] != 0 || o[2] < 1 || o[2] > kMaxSignal ||
        b.n + o[2] > kMaxPrologue)
      break;
    for (int i = 0; i < (int)o[2]; ++i) {
      b.ptr[b.n] = (unsigned*)o[5 + i];
      b.delta[b.n] = (int)o[4];
      ++b.n;
    }
  }
  return first;
}

}  // namespace ddlb
