// A layer's data gradient (DGRAD) and weight gradient (WGRAD) in ONE launch.
// Measured on the config-2 step (profiles/r02/dual_ab.txt): the 3-tap pairs
// interleaved, dec conv_in 109.0 -> 105.8 us and enc k3 66.1 -> 61.1 us per
// pair; the 1x1 pairs interleaved ran 8-20% slower, so by default they run in
// sequence inside the launch (DGRAD's round first), 0.7% off the step.
//
// Both read the same output gradient dy and are independent.  As two launches
// each is one round of 512 four-wave workgroups (two per CU) whose slots all
// reach the same phase together: the 1x1 DGRAD's fused GroupNorm/GLU-backward
// epilogue is an HBM burst every workgroup issues at once, and each launch
// pays its own ramp and tail.  Here the grid interleaves the two GEMMs'
// workgroups, 8 + 8 per 16 blocks, so each CU runs one workgroup of each:
// one's HBM-heavy epilogue runs beside the other's MFMA main loop, and one
// ramp and one tail cover both.  Each workgroup runs the unchanged kernel body
// (vqx_gemm_kernel.h conv_gemm_body / conv_tr_body / wgrad_tr_body) on its own
// tile grid; the branch is uniform per workgroup.
#include "vqx_gemm_inst.h"

namespace vqx {

// blockIdx -> (DGRAD?, workgroup index in that GEMM's grid): groups of
// ch DGRAD + ch WGRAD blocks (ch % 8 == 0) while both have workgroups left,
// then the rest of DGRAD, then the rest of WGRAD.  In the paired region the
// sub-index keeps blockIdx % 8 (the XCD), so each body's XCD-aware tile map
// still applies.
__device__ __forceinline__ bool dual_split(int b, int nd, int nw, int ch, int& sub) {
  const int m = (nd < nw ? nd : nw) / ch * ch;
  if (b < 2 * m) {
    const int g = b / (2 * ch), x = b - g * 2 * ch;
    sub = g * ch + (x < ch ? x : x - ch);
    return x < ch;
  }
  const int j = b - 2 * m;
  if (j < nd - m) {
    sub = m + j;
    return true;
  }
  sub = m + (j - (nd - m));
  return false;
}

constexpr int cmax(int a, int b) { return a > b ? a : b; }

// 1x1 layer: conv_gemm_kernel DGRAD (epilogue kind EKD) + conv_gemm_kernel
// WGRAD, DGRAD's workgroups first (one round), WGRAD's filling the slots they
// free (nd % 8 == 0 keeps the XCD map of both)
template <int EKD>
__global__ __launch_bounds__(256, 2) void dual_k1_kernel(GemmParams PD, GemmParams PW, int nd, int nw, int ch) {
  __shared__ __attribute__((aligned(16))) char smem[conv_gemm_smem<bf16_t, 64, 2>()];
  (void)ch;
  const int b = blockIdx.x;
  if (b < nd) conv_gemm_body<bf16_t, MODE_DGRAD, VQX_PRO_NONE, false, 64, 2, EKD>(PD, b, nd, smem);
  else conv_gemm_body<bf16_t, MODE_WGRAD, VQX_PRO_NONE, false, 64, 2, EK_NONE>(PW, b - nd, nw, smem);
}

// the same, three workgroups per CU (32-deep K-tiles in a 3-deep ring, 48 KiB
// of LDS): the automatic choice (POL_K1_2PCU keeps the two-per-CU kernel).
// The DGRAD round leaves a third of the slots free, which the WGRAD
// workgroups (or co-resident kernels) take at once.
template <int EKD>
__global__ __launch_bounds__(256, VQX_K1_OCC) void dual_k1_3_kernel(GemmParams PD, GemmParams PW, int nd, int nw,
                                                                     int ch) {
  __shared__ __attribute__((aligned(16))) char smem[conv_gemm_smem<bf16_t, VQX_K1_BK, VQX_K1_NST>()];
  (void)ch;
  const int b = blockIdx.x;
  if (b < nd) conv_gemm_body<bf16_t, MODE_DGRAD, VQX_PRO_NONE, false, VQX_K1_BK, VQX_K1_NST, EKD>(PD, b, nd, smem);
  else conv_gemm_body<bf16_t, MODE_WGRAD, VQX_PRO_NONE, false, VQX_K1_BK, VQX_K1_NST, EK_NONE>(PW, b - nd, nw, smem);
}

// 3-tap layer: conv_tr_kernel DGRAD (epilogue kind EKD) + wgrad_tr_kernel
template <int EKD>
__global__ __launch_bounds__(256, 2) void dual_tr_kernel(GemmParams PD, GemmParams PW, int nd, int nw, int ch) {
  __shared__ __attribute__((aligned(16))) char smem[cmax(conv_tr_smem<32>(), wgrad_tr_smem())];
  int sub;
  if (dual_split(blockIdx.x, nd, nw, ch, sub)) conv_tr_body<MODE_DGRAD, EKD, 32>(PD, sub, nd, smem);
  else wgrad_tr_body<EK_NONE>(PW, sub, nw, smem);
}

bool launch_dual(const GemmParams& PD, int nd, const GemmParams& PW, int nw, hipStream_t s) {
  if (PD.pro != VQX_PRO_NONE || PW.pro != VQX_PRO_NONE || nd <= 0 || nw <= 0) return false;
  const int ekd = pick_ek(PD.epi);
  const void* fn = nullptr;
  int kind = 0;
  if (tap_reuse_ok(PD, true, false) && tr8_segs(PD) == 0 && PD.kcin % 32 == 0) {
    if (PW.tap_reuse != 1) return false;
    kind = 2;
    switch (ekd) {
      case EK_NONE: fn = (const void*)dual_tr_kernel<EK_NONE>; break;
      case EK_ELEM: fn = (const void*)dual_tr_kernel<EK_ELEM>; break;
      case EK_COLSUM: fn = (const void*)dual_tr_kernel<EK_COLSUM>; break;
      default: return false;
    }
  } else if (PD.ntaps == 1 && PW.ntaps == 1 && PW.tap_reuse == 0 && nd % 8 == 0) {
    kind = 3;
    if (PD.policy == POL_AUTO) {
      kind = 4;
      switch (ekd) {
        case EK_NONE: fn = (const void*)dual_k1_3_kernel<EK_NONE>; break;
        case EK_ELEM: fn = (const void*)dual_k1_3_kernel<EK_ELEM>; break;
        case EK_COLSUM: fn = (const void*)dual_k1_3_kernel<EK_COLSUM>; break;
        case EK_GNBWD: fn = (const void*)dual_k1_3_kernel<EK_GNBWD>; break;
        default: return false;
      }
    } else {
      switch (ekd) {
        case EK_NONE: fn = (const void*)dual_k1_kernel<EK_NONE>; break;
        case EK_ELEM: fn = (const void*)dual_k1_kernel<EK_ELEM>; break;
        case EK_COLSUM: fn = (const void*)dual_k1_kernel<EK_COLSUM>; break;
        case EK_GNBWD: fn = (const void*)dual_k1_kernel<EK_GNBWD>; break;
        default: return false;
      }
    }
  } else {
    return false;
  }
  const double flops = 2.0 * (double)PD.n_rows * PD.Nc * PD.K + 2.0 * (double)PW.n_rows * PW.Mc * PW.Nc;
  // probe label: mode 3 = dual, prologue slot = kind (2: 3-tap, 3: 1x1 in sequence, 4: 1x1 three per CU), gen = 5
  const int info[5] = {VQX_BF16, 3, kind, 5, ekd};
  const int chunk = 256;  // interleave period: blocks of each GEMM per group (profiles/r02/chunk_probe.txt)
  GemmParams pd = PD, pw = PW;
  int a = nd, b = nw, c = chunk;
  void* args[] = {(void*)&pd, (void*)&pw, (void*)&a, (void*)&b, (void*)&c};
  gemm_launch_args(fn, nd + nw, s, args, info, flops, 256);
  return true;
}

}  // namespace vqx
