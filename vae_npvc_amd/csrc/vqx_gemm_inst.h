// Launch glue shared by the per-mode instantiation units (vqx_gemm_fwd.hip,
// vqx_gemm_dgrad.hip, vqx_gemm_wgrad.hip), split so hipcc builds them in
// parallel.  Pipeline variants of the bf16 GEMM (vqx_set_gemm_tile):
//   1: BK = 64, 2-deep LDS-DMA ring (default)
//   2: BK = 32, 4-deep ring (three K-tiles in flight; measured 5-30% slower on
//      every config-2 layer, kept for A/B runs)
// f32 (parity mode) always runs BK = 32, 2-deep.
#pragma once
#include "vqx_gemm_kernel.h"

namespace vqx {

// vqx_gemm.hip: plain launch, or the probe's event-stamped launch
void gemm_launch(const void* fn, int grid, hipStream_t s, const GemmParams& P, const int info[5], double flops);

template <typename T, int MODE, bool GEN, int BK, int NST>
void launch_variant(const GemmParams& P, int grid, hipStream_t s, int variant) {
  const double flops = MODE == MODE_WGRAD ? 2.0 * (double)P.n_rows * P.Mc * P.Nc
                                          : 2.0 * (double)P.n_rows * P.Nc * P.K;
  const int info[5] = {sizeof(T) == 2 ? VQX_BF16 : VQX_F32, MODE, P.pro, GEN ? 1 : 0, variant};
  const void* fn;
  if constexpr (MODE == MODE_DGRAD) {
    fn = (const void*)conv_gemm_kernel<T, MODE, VQX_PRO_NONE, GEN, BK, NST>;
  } else {
    switch (P.pro) {
      case VQX_PRO_NONE: fn = (const void*)conv_gemm_kernel<T, MODE, VQX_PRO_NONE, GEN, BK, NST>; break;
      case VQX_PRO_LRELU: fn = (const void*)conv_gemm_kernel<T, MODE, VQX_PRO_LRELU, GEN, BK, NST>; break;
      case VQX_PRO_RELU: fn = (const void*)conv_gemm_kernel<T, MODE, VQX_PRO_RELU, GEN, BK, NST>; break;
      default: fn = (const void*)conv_gemm_kernel<T, MODE, VQX_PRO_SCALE_RELU, GEN, BK, NST>; break;
    }
  }
  gemm_launch(fn, grid, s, P, info, flops);
}

template <int MODE>
void launch_mode_dt(const GemmParams& P, int grid, bool bf16, bool gen, int variant, hipStream_t s) {
  if (!bf16) {
    if (gen) launch_variant<float, MODE, true, 32, 2>(P, grid, s, 0);
    else launch_variant<float, MODE, false, 32, 2>(P, grid, s, 0);
    return;
  }
#define VQX_V(BK, NST)                                                  \
  if (gen) launch_variant<bf16_t, MODE, true, BK, NST>(P, grid, s, variant); \
  else launch_variant<bf16_t, MODE, false, BK, NST>(P, grid, s, variant);
  if (variant == 2) {
    VQX_V(32, 4)
  } else {
    VQX_V(64, 2)
  }
#undef VQX_V
}

}  // namespace vqx
