// gemm_f16: instantiations of the MFMA GEMM kernels (see gemm_mfma.hip).
#include "gemm_kernels.h"
#include "gemm_entry.h"

namespace ddlb {
hipError_t launch_fast_f16(const GemmArgs& p, int dout, int tile, hipStream_t s) {
  if (dout == DT_F16) return launch_cfg<MmaF16, DT_F16>(p, tile, s);
  if (dout == DT_F32) return launch_cfg<MmaF16, DT_F32>(p, tile, s);
  return hipErrorInvalidValue;
}
}  // namespace ddlb
