// GroupNorm(/GLU)-backward element math of the apply kernel (vqx_misc.hip
// gn_bwd_apply_vec_kernel), kept in one header so any other kernel applying it
// (the measured-and-rejected fused 1x1 DGRAD apply, tools/lab/
// dual_k1g_apply.patch) produces the same dx bit for bit.  Reference: autograd
// of layers.py 236-242 (tanh * sigmoid of the GroupNorm halves) and 170-176
// (GroupNorm).
#pragma once
#include "vqx_common.h"

namespace vqx {

// dL/dh (the GroupNorm output's gradient) and xhat for W channels of one frame.
//   glu: g = dL/d(tanh(h_a) * sigmoid(h_b)), ua / ub the GroupNorm inputs of
//        the two halves, mr4 = (mean_a, rstd_a, mean_b, rstd_b);
//   else: g = dL/dh, ua the GroupNorm input, mr4 = (mean, rstd).
// Every product/sum below is one rounding, fused only where written as fmaf
// (contraction off), so the two kernels agree bit for bit whatever the
// compiler's vectorisation of either.
template <typename T, int W>
__device__ __forceinline__ void gn_row_math(const float* g, const float* ua, const float* ub, bool glu,
                                            const float* mr4, const float* ga, const float* ba, const float* gb,
                                            const float* bb, float* dha, float* xa, float* dhb, float* xb) {
#pragma clang fp contract(off)
  if (!glu) {
#pragma unroll
    for (int i = 0; i < W; ++i) { dha[i] = g[i]; xa[i] = (ua[i] - mr4[0]) * mr4[1]; }
    return;
  }
#pragma unroll
  for (int i = 0; i < W; ++i) {
    const float xha = (ua[i] - mr4[0]) * mr4[1];
    const float xhb = (ub[i] - mr4[2]) * mr4[3];
    const float ha = fmaf(xha, ga[i], ba[i]);
    const float hb = fmaf(xhb, gb[i], bb[i]);
    constexpr bool FAST = sizeof(T) == 2;
    const float ta = fmaf(2.f, frcp<FAST>(1.f + __expf(-2.f * ha)), -1.f);  // tanh
    const float sb = frcp<FAST>(1.f + __expf(-hb));                          // sigmoid
    dha[i] = (g[i] * sb) * fmaf(-ta, ta, 1.f);
    dhb[i] = (g[i] * ta) * (sb * (1.f - sb));
    xa[i] = xha;
    xb[i] = xhb;
  }
}

// dL/du = rstd * (gamma * dh - m1 - xhat * m2), m1 = mean(gamma * dh),
// m2 = mean(gamma * dh * xhat) over the (utterance, group)
template <int W>
__device__ __forceinline__ void gn_dx(const float* dh, const float* xh, const float* ga, float rstd, float m1,
                                      float m2, float* o) {
#pragma clang fp contract(off)
#pragma unroll
  for (int i = 0; i < W; ++i) o[i] = rstd * fmaf(-xh[i], m2, fmaf(ga[i], dh[i], -m1));
}

}  // namespace vqx
