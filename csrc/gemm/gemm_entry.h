// Per-dtype launch entry points (one translation unit each), used by gemm_launch().
#pragma once
#include "gemm.h"

namespace ddlb {
hipError_t launch_fast_bf16(const GemmArgs& p, int dout, int tile, hipStream_t s);
hipError_t launch_fast_f16(const GemmArgs& p, int dout, int tile, hipStream_t s);
hipError_t launch_fast_fp8(const GemmArgs& p, int dout, int tile, hipStream_t s);
hipError_t launch_fast_f32(const GemmArgs& p, int dout, int tile, hipStream_t s);
hipError_t launch_fast_mx(const GemmArgs& p, int dout, int tile, hipStream_t s);
hipError_t launch_generic(const GemmArgs& p, int din, int dout, hipStream_t s);
}  // namespace ddlb
