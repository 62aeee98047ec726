// gemm_generic: instantiations of the MFMA GEMM kernels (see gemm_mfma.hip).
#include "gemm_kernels.h"
#include "gemm_entry.h"

namespace ddlb {
hipError_t launch_generic(const GemmArgs& p, int din, int dout, hipStream_t s) {
#define GEN(DI, DO) if (din == DI && dout == DO) return launch_generic_t<DI, DO>(p, s)
  GEN(DT_BF16, DT_BF16); GEN(DT_BF16, DT_F32); GEN(DT_F16, DT_F16); GEN(DT_F16, DT_F32);
  GEN(DT_F32, DT_F32); GEN(DT_F64, DT_F64); GEN(DT_FP8, DT_BF16); GEN(DT_FP8, DT_F16);
  GEN(DT_FP8, DT_F32);
#undef GEN
  return hipErrorInvalidValue;
}
}  // namespace ddlb
