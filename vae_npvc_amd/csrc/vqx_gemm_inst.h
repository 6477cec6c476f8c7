// Launch glue shared by the per-mode instantiation units (vqx_gemm_fwd.hip,
// vqx_gemm_dgrad.hip, vqx_gemm_wgrad.hip), split so hipcc builds them in
// parallel.  bf16 runs BK = 64 with a 2-deep LDS-DMA ring (BK = 32 with a
// 4-deep ring measured 5-30% slower on every config-2 layer:
// profiles/r01/gemm_lab.txt); f32 (parity mode) runs BK = 32, 2-deep.
//
// Instances: the bf16 fast path (no prologue, cin % 64 == 0) gets one kernel
// per epilogue kind (EK_*), and so does the tap-reuse kernel for 3-tap layers; prologues, GEN tiles (cin % BK != 0) and f32 use
// the generic EK_ALL kernel.  WGRAD's epilogue is the slab store (EK_NONE).
#pragma once
#include "vqx_gemm_kernel.h"
#include "vqx_gemm_pp.h"

namespace vqx {

// vqx_gemm.hip: plain launch, or the probe's event-stamped launch
void gemm_launch(const void* fn, int grid, hipStream_t s, const GemmParams& P, const int info[5], double flops,
                 int block = 256);
void gemm_launch_args(const void* fn, int grid, hipStream_t s, void** args, const int info[5], double flops,
                      int block = 256);

// vqx_gemm_dual.hip: one layer's data and weight gradients in ONE launch
// (dual_k1_kernel / dual_tr_kernel) where an instance covers the pair;
// false = not covered (the caller launches them separately)
bool launch_dual(const GemmParams& PD, int nd, const GemmParams& PW, int nw, hipStream_t s);

// Kernel policy of a call (vqx_conv_args.kernel_policy, include/vqx.h): 0
// automatic, 1 implicit-im2col kernels only (no tap reuse, no fused
// DGRAD + WGRAD launch), 2 / 3 the tall tap-reuse kernel with 256 / 512-frame
// tiles wherever it applies, 4 the 128-frame tap-reuse kernel only, 5 as
// automatic but the bf16 1x1 FWD / DGRAD+WGRAD on the two-workgroups-per-CU
// kernels (the round-4 choice).  Automatically a 1x1 grid of up to 3 x CUs
// tiles runs on the three-workgroups-per-CU kernels: one round with a third of
// the slots spare, which the fused WGRAD workgroups (and co-resident kernels,
// e.g. RCCL's) take (profiles/r05/policy_ab.txt: step -1.4%).
enum { POL_AUTO = 0, POL_IM2COL = 1, POL_TALL256 = 2, POL_TALL512 = 3, POL_TR128 = 4, POL_K1_2PCU = 5 };

// conv_tr_kernel applies: bf16, no prologue, 3 taps / pad 1, 32-channel K
// slices (16-channel slices when cin % 32 != 0, e.g. the 80-mel input conv),
// and every 128-frame tile inside one utterance
inline bool tap_reuse_ok(const GemmParams& P, bool bf16, bool gen) {
  return bf16 && P.pro == VQX_PRO_NONE && P.ntaps == 3 && P.pad == 1 && P.dil == 1 && P.kcin % 16 == 0 &&
         (!gen || P.kcin % 32 != 0) && P.K == 3 * P.kcin && P.T % 128 == 0 && P.n_rows % 128 == 0 &&
         P.policy != POL_IM2COL;
}

// wgrad_tr_kernel applies: bf16, no prologue, 3 taps / pad 1, c_dim % 64 == 0,
// 64-frame K-tiles inside one utterance
inline bool wgrad_tr_ok(int64_t n_rows, int T, int c_dim, int ntaps, int pad, int dil, bool bf16, int pro,
                        int policy) {
  return bf16 && pro == VQX_PRO_NONE && ntaps == 3 && pad == 1 && dil == 1 && c_dim % 64 == 0 && T % 64 == 0 &&
         n_rows % 64 == 0 && policy != POL_IM2COL;
}

// frame segments per conv_tr8_kernel tile (0 = use conv_tr_kernel).  Policy 2 /
// 3 forces 256 / 512 frames, 4 none.  Automatically the 512-frame tile where it
// still gives every CU a workgroup (config 2: dec_in FWD, 57 vs 61 us in the
// step); the 256-frame tile measured equal on enc FWD and 7-10% slower on both
// DGRADs (profiles/r02/tr_lab.txt), so it is never picked automatically.
inline int tr8_segs(const GemmParams& P) {
  if (P.T % 256 || P.kcin % 32) return 0;
  const int tn = (P.Nc + kBN - 1) / kBN;
  if (P.policy == POL_TR128) return 0;
  if (P.policy == POL_TALL256 || P.policy == POL_TALL512) {
    const int segs = P.policy == POL_TALL256 ? 1 : 2;
    return P.n_rows % (256 * segs) == 0 ? segs : 0;
  }
  if (P.n_rows % 512 == 0 && (P.n_rows / 512) * tn >= 256) return 2;
  return 0;
}

// Lab switch (build.py -D VQX_TR_FWD_LAB=n; 0 in the library): the automatic
// 3-tap FWD on the tall 256-frame kernel with a 3-deep (1) or 2-deep (2) ring
// of 32-channel stages instead of conv_tr_kernel's 128-frame tiles.
#ifndef VQX_TR_FWD_LAB
#define VQX_TR_FWD_LAB 0
#endif

template <int MODE, int EK>
void launch_tr(const GemmParams& P, int grid, hipStream_t s) {
  const double flops = 2.0 * (double)P.n_rows * P.Nc * P.K;
  if constexpr (MODE == MODE_FWD && VQX_TR_FWD_LAB != 0) {
    if (P.policy == POL_AUTO && tr8_segs(P) == 0 && P.T % 256 == 0 && P.n_rows % 256 == 0 && P.kcin % 32 == 0) {
      GemmParams Q = P;
      Q.tiles_m = (int)(P.n_rows / 256);
      const int info8[5] = {VQX_BF16, MODE, 1, 3, EK};
      const void* fn = VQX_TR_FWD_LAB == 1 ? (const void*)conv_tr8_kernel<MODE, EK, 1, 32, 3>
                                           : (const void*)conv_tr8_kernel<MODE, EK, 1, 32, 2>;
      gemm_launch(fn, Q.tiles_m * Q.tiles_n, s, Q, info8, flops, 512);
      return;
    }
  }
  if (const int segs = tr8_segs(P)) {
    GemmParams Q = P;
    Q.tiles_m = (int)(P.n_rows / (256 * segs));
    if (segs == 2) {  // gen = 6: conv_pp_kernel (ping-pong groups), prologue slot = SEGS
      const int infop[5] = {VQX_BF16, MODE, 2, 6, EK};
      gemm_launch((const void*)conv_pp_kernel<MODE, EK, 2, 2>, Q.tiles_m * Q.tiles_n, s, Q, infop, flops, 512);
      return;
    }
    const int info8[5] = {VQX_BF16, MODE, segs, 3, EK};  // gen = 3: conv_tr8_kernel, prologue slot = SEGS
    gemm_launch((const void*)conv_tr8_kernel<MODE, EK, 1>, Q.tiles_m * Q.tiles_n, s, Q, info8, flops, 512);
    return;
  }
  const int bkc = P.kcin % 32 == 0 ? 32 : 16;  // 16-channel stages (4-deep ring) only for cin % 32 != 0
  // gen = 2: tap-reuse kernel; the prologue slot carries the stage depth in channels
  const int info[5] = {VQX_BF16, MODE, bkc, 2, EK};
  if (bkc == 16) gemm_launch((const void*)conv_tr_kernel<MODE, EK, 16>, grid, s, P, info, flops);
  else gemm_launch((const void*)conv_tr_kernel<MODE, EK, 32>, grid, s, P, info, flops);
}

// smallest epilogue kind whose feature mask covers `epi`
inline int pick_ek(int epi) {
  for (int ek = EK_NONE; ek < EK_ALL; ++ek)
    if ((epi & ~ek_mask(ek)) == 0) return ek;
  return EK_ALL;
}

// tap-reuse FWD / DGRAD with the epilogue kind of P.epi
template <int MODE>
void dispatch_tr(const GemmParams& P, int grid, hipStream_t s) {
  switch (pick_ek(P.epi)) {
    case EK_NONE: launch_tr<MODE, EK_NONE>(P, grid, s); break;
    case EK_ELEM: launch_tr<MODE, EK_ELEM>(P, grid, s); break;
    case EK_GNADD: launch_tr<MODE, EK_GNADD>(P, grid, s); break;
    case EK_SPLIT: launch_tr<MODE, EK_SPLIT>(P, grid, s); break;
    case EK_COLSUM: launch_tr<MODE, EK_COLSUM>(P, grid, s); break;
    case EK_GNSTATS: launch_tr<MODE, EK_GNSTATS>(P, grid, s); break;
    case EK_GNBWD: launch_tr<MODE, EK_GNBWD>(P, grid, s); break;
    default: launch_tr<MODE, EK_ALL>(P, grid, s); break;
  }
}

// vqx_gemm.hip: compute units of the current device; true when a grid of
// three per CU fits one round (automatic policy), or a grid of 2-per-CU
// workgroups needs more than one round but at most 1.5 (POL_K1_2PCU)
int cu_count();
bool three_per_cu(int grid, int policy);

template <typename T, int MODE, int PRO, bool GEN, int EK>
void launch_one(const GemmParams& P, int grid, hipStream_t s) {
  constexpr int BK = sizeof(T) == 2 ? 64 : 32;
  const double flops = MODE == MODE_WGRAD ? 2.0 * (double)P.n_rows * P.Mc * P.Nc
                                          : 2.0 * (double)P.n_rows * P.Nc * P.K;
  if constexpr (sizeof(T) == 2 && !GEN && MODE != MODE_WGRAD && PRO == VQX_PRO_NONE &&
                (EK == EK_NONE || EK == EK_ELEM || EK == EK_SPLIT)) {
    // (not GNADD: its prefetched epilogue operands need the registers of the
    // two-per-CU kernel -- the encoder skip FWD ran 32.9 vs 27.6 us three per CU,
    // profiles/r05/rocprof_summary_gnadd3.txt, and 27.7 vs 25.2 us three per CU
    // without the prefetch, profiles/r05/k1_pipeline_ab.txt)
    // gen = 4: conv_gemm3_kernel (32-deep K-tiles, three workgroups per CU);
    // measured on the 1x1 640-column res/skip layers only, so 1x1 only
    if (P.ntaps == 1 && three_per_cu(grid, P.policy)) {
      const int info3[5] = {VQX_BF16, MODE, P.pro, 4, EK};
      gemm_launch((const void*)conv_gemm3_kernel<T, MODE, PRO, GEN, EK>, grid, s, P, info3, flops);
      return;
    }
  }
  const int info[5] = {sizeof(T) == 2 ? VQX_BF16 : VQX_F32, MODE, P.pro, GEN ? 1 : 0, EK};
  gemm_launch((const void*)conv_gemm_kernel<T, MODE, PRO, GEN, BK, 2, EK>, grid, s, P, info, flops);
}

template <typename T, int MODE, bool GEN, int EK>
void launch_pro(const GemmParams& P, int grid, hipStream_t s) {
  if constexpr (MODE == MODE_DGRAD) {
    launch_one<T, MODE, VQX_PRO_NONE, GEN, EK>(P, grid, s);
  } else {
    switch (P.pro) {
      case VQX_PRO_NONE: launch_one<T, MODE, VQX_PRO_NONE, GEN, EK>(P, grid, s); break;
      case VQX_PRO_LRELU: launch_one<T, MODE, VQX_PRO_LRELU, GEN, EK>(P, grid, s); break;
      case VQX_PRO_RELU: launch_one<T, MODE, VQX_PRO_RELU, GEN, EK>(P, grid, s); break;
      default: launch_one<T, MODE, VQX_PRO_SCALE_RELU, GEN, EK>(P, grid, s); break;
    }
  }
}

template <int MODE>
void launch_mode_dt(const GemmParams& P, int grid, bool bf16, bool gen, hipStream_t s) {
  constexpr int EKW = MODE == MODE_WGRAD ? EK_NONE : EK_ALL;  // generic epilogue of this mode
  if (!bf16) {
    if (gen) launch_pro<float, MODE, true, EKW>(P, grid, s);
    else launch_pro<float, MODE, false, EKW>(P, grid, s);
    return;
  }
  if (gen) {
    if constexpr (MODE != MODE_WGRAD) {  // 16-channel tap reuse (cin % 32 != 0, e.g. the 80-mel input conv)
      if (P.pro == VQX_PRO_NONE && tap_reuse_ok(P, bf16, gen)) {
        dispatch_tr<MODE>(P, grid, s);
        return;
      }
    }
    launch_pro<bf16_t, MODE, true, EKW>(P, grid, s);
    return;
  }
  if constexpr (MODE == MODE_WGRAD) {
    if (P.tap_reuse) {
      const double flops = 2.0 * (double)P.n_rows * P.Mc * P.Nc;
      // gen = 2: tap-reuse kernel (the prologue slot: 1 K group)
      const int info[5] = {VQX_BF16, MODE_WGRAD, 1, 2, EK_NONE};
      gemm_launch((const void*)wgrad_tr_kernel<EK_NONE>, grid, s, P, info, flops);
      return;
    }
    launch_pro<bf16_t, MODE, false, EK_NONE>(P, grid, s);
  } else {
    if (P.pro != VQX_PRO_NONE) {
      launch_pro<bf16_t, MODE, false, EK_ALL>(P, grid, s);
      return;
    }
    if (tap_reuse_ok(P, bf16, gen)) {
      dispatch_tr<MODE>(P, grid, s);
      return;
    }
    switch (pick_ek(P.epi)) {
      case EK_NONE: launch_one<bf16_t, MODE, VQX_PRO_NONE, false, EK_NONE>(P, grid, s); break;
      case EK_ELEM: launch_one<bf16_t, MODE, VQX_PRO_NONE, false, EK_ELEM>(P, grid, s); break;
      case EK_GNADD: launch_one<bf16_t, MODE, VQX_PRO_NONE, false, EK_GNADD>(P, grid, s); break;
      case EK_SPLIT: launch_one<bf16_t, MODE, VQX_PRO_NONE, false, EK_SPLIT>(P, grid, s); break;
      case EK_COLSUM: launch_one<bf16_t, MODE, VQX_PRO_NONE, false, EK_COLSUM>(P, grid, s); break;
      case EK_GNSTATS: launch_one<bf16_t, MODE, VQX_PRO_NONE, false, EK_GNSTATS>(P, grid, s); break;
      case EK_GNBWD: launch_one<bf16_t, MODE, VQX_PRO_NONE, false, EK_GNBWD>(P, grid, s); break;
      default: launch_one<bf16_t, MODE, VQX_PRO_NONE, false, EK_ALL>(P, grid, s); break;
    }
  }
}

}  // namespace vqx
