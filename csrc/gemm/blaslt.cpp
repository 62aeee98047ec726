// hipBLASLt backend for PLAIN GEMMs inside native plans (gemm_mode = blas).
//
// The hand-written kernels (gemm_kernels.h) stay the path for everything fused — arrival-flag
// gated tiles, epilogue activations, fp8/MX — and for ragged groupings; a plain or
// bf16/f16/f32 GEMM may instead run on the vendor library, which is what the
// reference's torch.matmul reaches (ddlb/primitives/TPColumnwise/pytorch.py:97). The autotuner
// (bench.py) times both and reports which one ran.
//
// Mapping to hipBLASLt's column-major problem: C[M,N] = A[M,K] * Bt[N,K]^T (all row-major) is
// C^T (N x M, ld = ldc) = op(Bt)^T-view (N x K) * A^T-view (K x M): "A" = Bt with TRANSA = T,
// "B" = A with TRANSB = N. Grouped-row addressing is not sent here (blaslt_supports).
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>

#include "gemm.h"

namespace ddlb {
namespace {

struct LtKey {
  int dev, din, dout;
  int64_t m, n, k, lda, ldb, ldc, batch, sa, sc;
  bool operator==(const LtKey& o) const { return std::memcmp(this, &o, sizeof(LtKey)) == 0; }
};
struct LtKeyHash {
  size_t operator()(const LtKey& k) const {
    const uint64_t* w = reinterpret_cast<const uint64_t*>(&k);
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < sizeof(LtKey) / 8; ++i) h = (h ^ w[i]) * 1099511628211ull;
    return (size_t)h;
  }
};
constexpr int kMaxAlgos = 16, kTuneReps = 10;
struct LtPlan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  bool ok = false, tuned = false;
  int ncand = 0, chosen = 0;
  hipblasLtMatmulHeuristicResult_t cands[kMaxAlgos];
};

// DDLB_BLAS_TUNE=0 keeps the heuristic's first choice (default: time the top candidates).
bool tune_enabled() {
  const char* v = std::getenv("DDLB_BLAS_TUNE");
  return v == nullptr || std::strcmp(v, "0") != 0;
}
// One handle per device; one workspace per (device, stream): two hipBLASLt GEMMs enqueued on
// different streams may run concurrently, so they must never share scratch memory.
struct LtDevice {
  hipblasLtHandle_t handle = nullptr;
  size_t ws_bytes = 0;  // the same cap for every stream's workspace
  std::unordered_map<hipStream_t, void*> workspace;
};

constexpr size_t kWorkspace = 64ull << 20;
std::mutex g_mu;
std::unordered_map<int, LtDevice> g_dev;
std::unordered_map<LtKey, LtPlan, LtKeyHash> g_plans;

// Workspace of stream ``s`` (allocated on first use; nullptr + 0 bytes if that fails, which
// restricts the plan to workspace-free algorithms).
void* workspace_for(LtDevice* d, hipStream_t s, size_t* bytes) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = d->workspace.find(s);
  if (it == d->workspace.end()) {
    void* w = nullptr;
    if (d->ws_bytes && hipMalloc(&w, d->ws_bytes) != hipSuccess) {
      (void)hipGetLastError();
      w = nullptr;
    }
    it = d->workspace.emplace(s, w).first;
  }
  *bytes = it->second ? d->ws_bytes : 0;
  return it->second;
}

bool lt_type(int dt, hipDataType* t) {
  switch (dt) {
    case DT_BF16: *t = HIP_R_16BF; return true;
    case DT_F16: *t = HIP_R_16F; return true;
    case DT_F32: *t = HIP_R_32F; return true;
    default: return false;
  }
}

LtDevice* device_state(int dev) {
  LtDevice& d = g_dev[dev];
  if (d.handle == nullptr) {
    if (hipblasLtCreate(&d.handle) != HIPBLAS_STATUS_SUCCESS) {
      d.handle = nullptr;
      return nullptr;
    }
    d.ws_bytes = kWorkspace;
  }
  return &d;
}

bool build_plan(LtDevice* d, const LtKey& key, LtPlan* pl) {
  hipDataType tin, tout;
  if (!lt_type(key.din, &tin) || !lt_type(key.dout, &tout)) return false;
  if (hipblasLtMatmulDescCreate(&pl->op, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS)
    return false;
  const int32_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(pl->op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(pl->op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  // column-major: "A" = Bt viewed K x N (ld = ldb), "B" = A viewed K x M (ld = lda), C: N x M
  if (hipblasLtMatrixLayoutCreate(&pl->la, tin, key.k, key.n, key.ldb) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&pl->lb, tin, key.k, key.m, key.lda) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&pl->lc, tout, key.n, key.m, key.ldc) != HIPBLAS_STATUS_SUCCESS)
    return false;
  if (key.batch > 1) {
    const int32_t b = (int32_t)key.batch;
    const int64_t s0 = 0, sa = key.sa, sc = key.sc;
    hipblasLtMatrixLayoutSetAttribute(pl->la, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &b, sizeof(b));
    hipblasLtMatrixLayoutSetAttribute(pl->la, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &s0,
                                      sizeof(s0));
    hipblasLtMatrixLayoutSetAttribute(pl->lb, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &b, sizeof(b));
    hipblasLtMatrixLayoutSetAttribute(pl->lb, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &sa,
                                      sizeof(sa));
    hipblasLtMatrixLayoutSetAttribute(pl->lc, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &b, sizeof(b));
    hipblasLtMatrixLayoutSetAttribute(pl->lc, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &sc,
                                      sizeof(sc));
  }
  hipblasLtMatmulPreference_t pref = nullptr;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return false;
  const uint64_t wsb = d->ws_bytes;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb,
                                        sizeof(wsb));
  int n = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(
      d->handle, pl->op, pl->la, pl->lb, pl->lc, pl->lc, pref, kMaxAlgos, pl->cands, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS) return false;
  for (int i = 0; i < n; ++i)  // keep the usable candidates, heuristic order
    if (pl->cands[i].state == HIPBLAS_STATUS_SUCCESS && pl->cands[i].workspaceSize <= d->ws_bytes)
      pl->cands[pl->ncand++] = pl->cands[i];
  if (pl->ncand == 0) return false;
  pl->algo = pl->cands[0].algo;
  pl->ws = pl->cands[0].workspaceSize;
  return true;
}

// Time the heuristic's top candidates on stream ``s`` with the real operands and keep the
// fastest (the top-1 heuristic is not always the fastest kernel for tall-skinny shapes). Runs
// once per shape, outside graph capture, with a host wait on an event: plans call it at bind
// time (PlanExecutor::prepare), never while enqueueing a run. C is overwritten.
void autotune(LtDevice* d, LtPlan* pl, const GemmArgs& p, hipStream_t s) {
  pl->tuned = true;
  if (pl->ncand < 2 || !tune_enabled()) return;
  size_t wsb = 0;
  void* ws = workspace_for(d, s, &wsb);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return;
  if (hipEventCreate(&e1) != hipSuccess) { hipEventDestroy(e0); return; }
  const float alpha = 1.f, beta = 0.f;
  float best = 1e30f;
  int best_i = 0;
  for (int i = 0; i < pl->ncand; ++i) {
    if (pl->cands[i].workspaceSize > wsb) continue;
    auto run = [&]() {
      return hipblasLtMatmul(d->handle, pl->op, &alpha, p.b, pl->la, p.a, pl->lb, &beta, p.c,
                             pl->lc, p.c, pl->lc, &pl->cands[i].algo, ws,
                             pl->cands[i].workspaceSize, s);
    };
    bool ok = true;
    for (int w = 0; w < 2 && ok; ++w) ok = run() == HIPBLAS_STATUS_SUCCESS;
    if (!ok) continue;
    hipEventRecord(e0, s);
    for (int r = 0; r < kTuneReps; ++r) run();
    hipEventRecord(e1, s);
    if (hipEventSynchronize(e1) != hipSuccess) break;
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) { best = ms; best_i = i; }
  }
  (void)hipGetLastError();
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  pl->algo = pl->cands[best_i].algo;
  pl->ws = pl->cands[best_i].workspaceSize;
  pl->chosen = best_i;
}

}  // namespace

bool blaslt_supports(const GemmArgs& p, int din, int dout) {
  hipDataType t;
  if (!lt_type(din, &t) || !lt_type(dout, &t)) return false;
  if (p.flags != nullptr || p.act != ACT_NONE || p.tile_order != 0 || p.a_table ||
      p.c_table)
    return false;
  if (p.M <= 0 || p.N <= 0 || p.K <= 0) return false;
  // Plain GEMMs only. Grouped-row (pipeline-stage) addressing stays on the MFMA kernels, which
  // read the grouped rows natively in one launch: the equivalent hipBLASLt strided batch with a
  // broadcast (stride-0) weight returned wrong tiles and then faulted on MI355X at the flagship
  // stage shapes (65536x1024x1024 split d=2..8, s=4; scripts/diag_blas_batch.py), while the
  // same call passed at small shapes.
  const int64_t ag = p.a_grp > 0 ? p.a_grp : p.M, cg = p.c_grp > 0 ? p.c_grp : p.M;
  if (ag != p.M || cg != p.M) return false;
  return true;
}

namespace {
// The cached (and, on first use with ``tune``, autotuned) plan of p's shape; nullptr if
// hipBLASLt cannot run it.
LtPlan* plan_for(const GemmArgs& p, int din, int dout, hipStream_t s, bool tune, LtDevice** dev_out) {
  if (!blaslt_supports(p, din, dout)) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  const int64_t grp = p.a_grp > 0 ? p.a_grp : p.M;
  LtKey key;
  std::memset(&key, 0, sizeof(key));
  key.dev = dev; key.din = din; key.dout = dout;
  key.m = grp; key.n = p.N; key.k = p.K;
  key.lda = p.lda; key.ldb = p.ldb; key.ldc = p.ldc;
  key.batch = p.M / grp;
  key.sa = (p.a_gstride > 0 ? p.a_gstride : grp) * p.lda;
  key.sc = (p.c_gstride > 0 ? p.c_gstride : grp) * p.ldc;
  LtDevice* d;
  LtPlan* pl;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    d = device_state(dev);
    if (d == nullptr) return nullptr;
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
      LtPlan fresh;
      fresh.ok = build_plan(d, key, &fresh);
      it = g_plans.emplace(key, fresh).first;
    }
    pl = &it->second;
  }
  if (!pl->ok) return nullptr;
  if (tune && !pl->tuned) autotune(d, pl, p, s);
  *dev_out = d;
  return pl;
}
}  // namespace

hipError_t blaslt_prepare(const GemmArgs& p, int din, int dout, hipStream_t s) {
  LtDevice* d = nullptr;
  if (plan_for(p, din, dout, s, true, &d) == nullptr) return hipErrorNotSupported;
  size_t wsb = 0;
  (void)workspace_for(d, s, &wsb);  // allocated now, not inside a later graph capture
  return hipSuccess;
}

hipError_t blaslt_gemm(const GemmArgs& p, int din, int dout, hipStream_t s) {
  // direct callers (ops.gemm) tune on first use; plans were tuned at bind time (prepare)
  LtDevice* d = nullptr;
  LtPlan* pl = plan_for(p, din, dout, s, true, &d);
  if (pl == nullptr) return hipErrorNotSupported;
  size_t wsb = 0;
  void* ws = workspace_for(d, s, &wsb);
  if (pl->ws > wsb) return hipErrorNotSupported;
  const float alpha = 1.f, beta = 0.f;
  const hipblasStatus_t st =
      hipblasLtMatmul(d->handle, pl->op, &alpha, p.b, pl->la, p.a, pl->lb, &beta, p.c, pl->lc,
                      p.c, pl->lc, &pl->algo, ws, pl->ws, s);
  return st == HIPBLAS_STATUS_SUCCESS ? hipSuccess : hipErrorLaunchFailure;
}

}  // namespace ddlb
