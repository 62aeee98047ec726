// GEMM lab: the product's persistent pt4 kernel (csrc/gemm/gemm_kernels.h, copied and optionally
// text-patched by research/lab/pt4_ablate.py into build/lab/<variant>/) as a standalone shared
// object, so several variants can be timed interleaved in ONE process (cdna guide §5.4 rule 24)
// without adding ablation switches to the product kernel. Plain rows, dense C, bf16 or MX-fp8 in,
// bf16 out. `dbg` is handed to the kernel as GemmArgs::timeout_word (unused by the ungated
// kernel): stamp variants write their s_memtime records there.
#include "gemm_kernels.h"

extern "C" int lab_pt4(const void* a, const void* b, void* c, int M, int N, int K, int mx,
                       void* dbg, void* stream) {
  ddlb::GemmArgs p;
  p.a = a;
  p.b = b;
  p.c = c;
  p.lda = K;
  p.ldb = K;
  p.ldc = N;
  p.M = M;
  p.N = N;
  p.K = K;
  p.a_grp = p.a_gstride = p.c_grp = p.c_gstride = M;
  p.timeout_word = (unsigned*)dbg;
  const hipStream_t s = (hipStream_t)stream;
  const int esz = mx ? 1 : 2;
  if (!ddlb::pt4_ok(p, esz) || !ddlb::c_fits_wt(p, 2)) return -1;
  const hipError_t e = mx ? ddlb::launch_pt4<ddlb::MmaMX, ddlb::DT_BF16>(p, s)
                          : ddlb::launch_pt4<ddlb::MmaBF16, ddlb::DT_BF16>(p, s);
  return (int)e;
}
