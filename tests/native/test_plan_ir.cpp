// Host-only check of the plan executor's IR half (csrc/runtime/plan_ir.h), built with
// AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_native_host.py, which feeds it the
// encoded op arrays of every plan the simulator tests build (fake, non-null addresses).
//
// Input file: int64 words  [nplans] then per plan [nstreams, nevents, nwords, words...].
// Per plan it validates the ops, decodes every GEMM, computes the graph-capture decision (RCCL /
// externally gated GEMM / side-stream cycle) and the fused replay prologue, prints one summary
// line, and checks that corrupted copies of the plan are refused (wrong length, a stream or
// event index out of range, an unknown kind, a count past the op size, a null operand).
#include <stdio.h>
#include <stdlib.h>

#include <fstream>
#include <string>
#include <vector>

#include "runtime/plan_ir.h"

using namespace ddlb;

static int failures = 0;
#define CHECK(cond, msg)                                       \
  do {                                                         \
    if (!(cond)) {                                             \
      fprintf(stderr, "FAIL plan %zu: %s\n", pi, (msg));       \
      ++failures;                                              \
    }                                                          \
  } while (0)

static bool refused(const std::vector<int64_t>& ops, size_t ns, size_t ne) {
  try {
    validate_ops(ops, ns, ne);
  } catch (const std::runtime_error&) {
    return true;
  }
  return false;
}

int main(int argc, char** argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: %s plans.bin\n", argv[0]);
    return 2;
  }
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<int64_t> all;
  int64_t w;
  while (f.read(reinterpret_cast<char*>(&w), sizeof w)) all.push_back(w);
  size_t pos = 0;
  auto next = [&]() -> int64_t {
    if (pos >= all.size()) {
      fprintf(stderr, "truncated input\n");
      exit(2);
    }
    return all[pos++];
  };
  const int64_t nplans = next();
  for (size_t pi = 0; pi < (size_t)nplans; ++pi) {
    const size_t ns = (size_t)next(), ne = (size_t)next(), nw = (size_t)next();
    std::vector<int64_t> ops(nw);
    for (size_t i = 0; i < nw; ++i) ops[i] = next();
    try {
      validate_ops(ops, ns, ne);
    } catch (const std::runtime_error& e) {
      fprintf(stderr, "FAIL plan %zu refused: %s\n", pi, e.what());
      ++failures;
      continue;
    }
    const std::vector<bool> used = used_streams(ops, ns);
    int nused = 0;
    for (bool u : used) nused += u;
    const bool unc = has_uncapturable_op(ops), cyc = side_stream_cycle(ops, ns, ne);
    BumpSignalArgs b;
    const size_t pro = fused_prologue(ops, b);
    CHECK(pro % kOpWords == 0 && pro <= ops.size() && b.n <= kMaxPrologue, "prologue bounds");
    printf("plan %zu ops %zu streams %d uncapturable %d cycle %d prologue %zu/%d", pi,
           ops.size() / kOpWords, nused, (int)unc, (int)cyc, pro / kOpWords, b.n);
    for (size_t i = 0; i < ops.size(); i += kOpWords) {
      if (ops[i] != OP_GEMM) continue;
      const GemmArgs g = decode_gemm(&ops[i]);
      CHECK(g.M >= 0 && g.N >= 0 && g.K > 0 && g.ksplit >= 1 && g.nsub >= 1 && g.nshards >= 1,
            "decoded GEMM fields");
      printf(" gemm %d %d %d %d %d %d %d %d", g.M, g.N, g.K, g.ksplit, g.ag_ctas, g.nsub,
             g.reserve_cus, (int)(g.flags != nullptr));
    }
    printf("\n");
    // corruptions must be refused
    if (!ops.empty()) {
      std::vector<int64_t> bad(ops.begin(), ops.end() - 1);
      CHECK(refused(bad, ns, ne), "truncated array accepted");
      bad = ops;
      bad[1] = (int64_t)ns;
      CHECK(refused(bad, ns, ne), "stream index out of range accepted");
      bad = ops;
      bad[0] = kLastOpKind + 1;
      CHECK(refused(bad, ns, ne), "unknown kind accepted");
      for (size_t i = 0; i < ops.size(); i += kOpWords) {
        bad = ops;
        int64_t* o = &bad[i];
        bool corrupt = true;
        switch (o[0]) {
          case OP_RECORD: case OP_WAIT: o[2] = (int64_t)ne; break;
          case OP_GEMM: o[3] = 0; break;
          case OP_SIGNAL: case OP_WAIT_SIGNAL: o[2] = kMaxSignal + 1; break;
          case OP_COPY_MULTI: case OP_COPY_BATCH: o[2] = kMaxCopySeg + 1; break;
          case OP_REDUCE: o[5] = kMaxReduceSrc + 1; break;
          case OP_COPY: o[2] = 0; break;
          default: corrupt = false;
        }
        if (corrupt) CHECK(refused(bad, ns, ne), "corrupted op accepted");
      }
    }
  }
  if (pos != all.size()) {
    fprintf(stderr, "trailing words in input\n");
    return 2;
  }
  printf("plan ir %s: %lld plans\n", failures ? "FAILED" : "ok", (long long)nplans);
  return failures ? 1 : 0;
}
