// Per-(input, output)-dtype launch entry points (one translation unit each), used by
// gemm_launch() in gemm_mfma.hip.
#pragma once
#include "gemm.h"

namespace ddlb {
hipError_t launch_fast_bf16_bf16(const GemmArgs& p, int tile, hipStream_t s);
hipError_t launch_fast_bf16_f32(const GemmArgs& p, int tile, hipStream_t s);
hipError_t launch_fast_f16_f16(const GemmArgs& p, int tile, hipStream_t s);
hipError_t launch_fast_f16_f32(const GemmArgs& p, int tile, hipStream_t s);
hipError_t launch_fast_fp8_bf16(const GemmArgs& p, int tile, hipStream_t s);
hipError_t launch_fast_fp8_f16(const GemmArgs& p, int tile, hipStream_t s);
hipError_t launch_fast_fp8_f32(const GemmArgs& p, int tile, hipStream_t s);
hipError_t launch_fast_f32_f32(const GemmArgs& p, int tile, hipStream_t s);
hipError_t launch_fast_mx(const GemmArgs& p, int dout, int tile, hipStream_t s);
hipError_t launch_generic(const GemmArgs& p, int din, int dout, hipStream_t s);

// Dispatch of the fast (MFMA) family by dtype pair; hipErrorInvalidValue if not provided.
inline hipError_t launch_fast(const GemmArgs& p, int din, int dout, int tile, hipStream_t s) {
  if (din == DT_BF16 && dout == DT_BF16) return launch_fast_bf16_bf16(p, tile, s);
  if (din == DT_BF16 && dout == DT_F32) return launch_fast_bf16_f32(p, tile, s);
  if (din == DT_F16 && dout == DT_F16) return launch_fast_f16_f16(p, tile, s);
  if (din == DT_F16 && dout == DT_F32) return launch_fast_f16_f32(p, tile, s);
  if (din == DT_FP8 && dout == DT_BF16) return launch_fast_fp8_bf16(p, tile, s);
  if (din == DT_FP8 && dout == DT_F16) return launch_fast_fp8_f16(p, tile, s);
  if (din == DT_FP8 && dout == DT_F32) return launch_fast_fp8_f32(p, tile, s);
  if (din == DT_F32 && dout == DT_F32) return launch_fast_f32_f32(p, tile, s);
  return hipErrorInvalidValue;
}
}  // namespace ddlb
