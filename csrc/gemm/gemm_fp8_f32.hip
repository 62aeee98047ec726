// gemm_fp8_f32: instantiations of the MFMA GEMM kernels for one (input, output) dtype pair, one
// translation unit per pair so the heavy kernel templates compile in parallel (see gemm_mfma.hip).
#include "gemm_kernels.h"
#include "gemm_entry.h"

namespace ddlb {
hipError_t launch_fast_fp8_f32(const GemmArgs& p, int tile, hipStream_t s) {
  return launch_cfg<MmaFP8, DT_F32>(p, tile, s);
}
}  // namespace ddlb
