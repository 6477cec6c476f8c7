// Conv1d / ConvTranspose1d (stride 1) as implicit-im2col GEMMs on gfx950 MFMA.
//
// One kernel template covers the three products of a conv layer:
//   FWD   Y[n][co]      = sum_{j,ci} pro(x[n+j*d-pad][ci]) * We[co][j][ci]
//   DGRAD Y[n][ci]      = sum_{j,co} dy[n+j*d-pad][co]     * We[co][k-1-j][ci]
//   WGRAD S[r][j*cd+c]  = sum_n      p[n][r]               * pro(q[n+s(j*d-pad)][c])
// (d = dilation; up to 8 taps)
// Frames (n = b*T + t) are the long GEMM dimension: 16,384 at config 2.
//
// Workgroup: 256 threads, 128x128 output tile, 4 waves in 2x2, each wave a
// 64x64 sub-tile = 2x2 MFMA blocks of 32x32, two workgroups per CU.  bf16:
// v_mfma_f32_32x32x16_bf16, BK = 32 or 64; f32 (parity mode):
// v_mfma_f32_32x32x2_f32, BK = 32, an exact fp32 fmaf chain.
//
// Staging: LDS-DMA (buffer_load ... lds) through an NST-deep ring of K-tiles
// (see conv_gemm_kernel).  Loads are raw buffer loads: an offset past the
// descriptor's range returns zeros, which is how the im2col zero padding at
// utterance edges, the ragged M/N edges and the K tail are produced without
// branches.  When a K-tile lies inside one tap (cin % BK == 0: every large
// layer) the tap shift and the channel offset are folded into a scalar byte
// shift, so the per-chunk VALU work is one select.  K-contiguous operands
// live K-major in LDS (ds_read_b128, XOR swizzle); K-strided operands
// (weights in DGRAD, both operands in WGRAD) are stored as they lie in memory
// and read with ds_read_b64_tr_b16 (bf16) or ds_read_b32 (f32).
//
// The MFMA's first operand is the one whose index is contiguous in the output
// (channels for FWD/DGRAD, j*cd+c for WGRAD), so each lane ends up holding 4
// consecutive output elements per register group: the epilogue does vector
// loads/stores (8 B bf16, 16 B f32) for bias, residual, masks and results.
#pragma once
#include <type_traits>
#include <utility>

#include "vqx_common.h"


namespace vqx {

constexpr int kBN = 128;  // tile width (and height)
constexpr unsigned kOOB = 0x80000000u;  // buffer offset that is always out of range -> loads 0
enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

// f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>): loop bodies
// whose index must be a compile-time constant before inlining-time SROA
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

struct GemmParams {
  const void* a;   // FWD/DGRAD: activation [N][lda]   WGRAD: p [N][lda]
  const void* b;   // FWD/DGRAD: packed We [cout_f][ntaps*cin_f]   WGRAD: q [N][ldb]
  int64_t a_bytes, b_bytes;
  int64_t n_rows;  // frames
  int T, lda, ldb;
  int kcin;        // FWD/DGRAD: channels per tap on the K side
  int K;           // FWD/DGRAD: ntaps*kcin
  int Mc, Nc;      // output dims: FWD/DGRAD rows = frames, cols = channels; WGRAD rows = r, cols = j*cd+c
  int ntaps, pad, sign;
  int dil;         // tap spacing in frames (dilation), >= 1
  int cdim;        // DGRAD: cin of the forward layer (= Nc); WGRAD: c_dim
  int pro;
  float pro_scale;
  int tiles_m, tiles_n, splits;
  int64_t k_per_split;
  // epilogue
  void* y;
  int ldy, epi, out_f32;
  const float* bias;
  const float* rowbias;
  const void* res;
  int ldres;
  const void* mask;
  int ldmask;
  float mask_slope, mask_scale;
  const void* gn_h;
  int ldgn;
  const float* gn_mr;
  const float* gn_gamma;
  const float* gn_beta;
  float* out2;
  int ldo2, split_col, out2_acc;
  void* y2;
  int ldy2, epi_act;
  float* colsum_part;
  float* stat_part;  // GNSTATS / GNBWD per-(128-row group, column tile) partials
  int gn_groups, gn_glu;
  int tap_reuse;   // WGRAD: 1 = wgrad_tr_kernel tiling (tiles_n counts 64-channel blocks of c)
  int slab_bf16;   // WGRAD: slabs stored as bf16 (bf16 operands only)
  const float* gn_tiles;  // GNADD: merge mean/rstd from these GNSTATS tiles (G = 1) and write gn_mr
  float gn_eps;
  int policy;      // host side: the call's kernel_policy (vqx_conv_args / vqx_wgrad_args)
  float* fix_dw;           // WGRAD (tap reuse, bf16 slabs): in-launch split-K reduction target, or null
  unsigned* fix_cnt;       // ... its per-tile arrival counters (left zero)
};

template <typename T> struct Cfg;
template <> struct Cfg<bf16_t> { static constexpr int EPC = 8, MNCPR = 16; };
template <> struct Cfg<float> { static constexpr int EPC = 4, MNCPR = 32; };

__device__ __forceinline__ float apply_pro(float v, int pro, float s) {
  if (pro == VQX_PRO_LRELU) return v > 0.f ? v : 0.2f * v;
  if (pro == VQX_PRO_RELU) return v > 0.f ? v : 0.f;
  if (pro == VQX_PRO_SCALE_RELU) { v = v * s; return v > 0.f ? v : 0.f; }
  return v;
}

template <typename T, int PRO>
__device__ __forceinline__ uint4 pro_chunk(uint4 u, float s) {
  if constexpr (PRO == VQX_PRO_NONE) {
    return u;
  } else if constexpr (sizeof(T) == 2) {
    unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float lo = __uint_as_float(w[i] << 16), hi = __uint_as_float(w[i] & 0xffff0000u);
      lo = apply_pro(lo, PRO, s);
      hi = apply_pro(hi, PRO, s);
      w[i] = pack_bf16x2(lo, hi);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    float f[4] = {__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = apply_pro(f[i], PRO, s);
    return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
  }
}

// tap of K index k when each tap spans c channels (ntaps <= 8)
__device__ __forceinline__ int tap_of(int k, int c, int nt) {
  if (nt <= 3) return (k >= c) + (k >= 2 * c);
  int j = 0;
#pragma unroll
  for (int t = 1; t < 8; ++t) j += (t < nt && k >= t * c) ? 1 : 0;
  return j;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_at(const void* base, int64_t shift_bytes, int64_t total_bytes) {
  int64_t rec = total_bytes - shift_bytes;
  if (rec < 0) rec = 0;
  if (rec > 0x7fffffff) rec = 0x7fffffff;
  return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + shift_bytes), (short)0, (int)rec, 0x00020000);
}

__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// LDS byte offsets of a 16-B chunk.  K-major rows hold KCH chunks (128-B
// rows: KCH = 8, 64-B rows: KCH = 4); the swizzle makes each 16-lane group of
// a 32x32 fragment's ds_read_b128 (rows {0-3,12-15,20-27} / {4-11,16-19,28-31},
// one chunk column) hit all 64 banks once.
template <int KCH>
__device__ __forceinline__ int kswz(int row) {
  if constexpr (KCH == 8) return (row >> 1) & 7;
  else return (row >> 2) & 3;
}
template <int KCH>
__device__ __forceinline__ int kmaj_off(int row, int ch) { return row * (16 * KCH) + 16 * (ch ^ kswz<KCH>(row)); }
__device__ __forceinline__ int mn_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
template <typename T>
__device__ __forceinline__ int mnmaj_off(int row, int ch) {
  if constexpr (sizeof(T) == 2) return row * 256 + 16 * (ch ^ mn_swz(row));
  else return row * 512 + 16 * ch;
}

// 8 consecutive elements (16 B bf16 / 32 B f32) at p+i
template <typename T>
__device__ __forceinline__ void ld8(const void* p, int64_t i, float* f) {
  if constexpr (sizeof(T) == 2) {
    const uint4 u = *(const uint4*)((const bf16_t*)p + i);
    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[2 * k] = __uint_as_float(w[k] << 16);
      f[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  } else {
    const f32x4_t a = *(const f32x4_t*)((const float*)p + i);
    const f32x4_t b = *(const f32x4_t*)((const float*)p + i + 4);
#pragma unroll
    for (int k = 0; k < 4; ++k) { f[k] = a[k]; f[4 + k] = b[k]; }
  }
}
template <typename T>
__device__ __forceinline__ void st8(void* p, int64_t i, const float* f) {
  if constexpr (sizeof(T) == 2) {
    uint4 u;
    u.x = pack_bf16x2(f[0], f[1]);
    u.y = pack_bf16x2(f[2], f[3]);
    u.z = pack_bf16x2(f[4], f[5]);
    u.w = pack_bf16x2(f[6], f[7]);
    *(uint4*)((bf16_t*)p + i) = u;
  } else {
    const f32x4_t a = {f[0], f[1], f[2], f[3]}, b = {f[4], f[5], f[6], f[7]};
    *(f32x4_t*)((float*)p + i) = a;
    *(f32x4_t*)((float*)p + i + 4) = b;
  }
}

// Optional streaming (non-temporal) stores of the output tile.  They make the
// producing GEMM 10-18% faster on the 1x1 layers in isolation
// (profiles/r01/gemm_lab.txt) but the whole step 1.3% (outputs) / 2.9% (also
// the WGRAD slabs) slower: the consumer then reads from HBM instead of the
// Infinity Cache (profiles/r01/nt_store_ab.txt).  Off by default.
template <typename T, bool NT = true>
__device__ __forceinline__ void st8_nt(void* p, int64_t i, const float* f) {
  if constexpr (!NT) {
    st8<T>(p, i, f);
    return;
  }
  typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
  if constexpr (sizeof(T) == 2) {
    const u32x4v u = {pack_bf16x2(f[0], f[1]),
                      pack_bf16x2(f[2], f[3]),
                      pack_bf16x2(f[4], f[5]),
                      pack_bf16x2(f[6], f[7])};
    __builtin_nontemporal_store(u, (u32x4v*)((bf16_t*)p + i));
  } else {
    const f32x4_t a = {f[0], f[1], f[2], f[3]}, b = {f[4], f[5], f[6], f[7]};
    __builtin_nontemporal_store(a, (f32x4_t*)((float*)p + i));
    __builtin_nontemporal_store(b, (f32x4_t*)((float*)p + i + 4));
  }
}

// Epilogue kinds: each conv_gemm_kernel instance compiles only the epilogue
// features of its kind (the runtime flags are masked with it), so the common
// launches do not carry the code of every fused epilogue (a 14k-instruction
// kernel body measured ~2 us slower per launch than a specialised one).
enum {
  EK_NONE = 0,     // store only (OUTF32 allowed)
  EK_ELEM = 1,     // BIAS | ROWBIAS | MASK | RES | ACT | ACT2 | OUTF32
  EK_GNADD = 2,    // ELEM + GNADD
  EK_SPLIT = 3,    // ELEM + SPLIT
  EK_COLSUM = 4,   // ELEM + COLSUM
  EK_GNSTATS = 5,  // ELEM + GNSTATS
  EK_GNBWD = 6,    // ELEM + COLSUM + GNBWD
  EK_ALL = 7       // every flag (generic path: prologues, GEN tiles, f32)
};
constexpr int kEpiElem = VQX_EPI_BIAS | VQX_EPI_ROWBIAS | VQX_EPI_MASK | VQX_EPI_RES | VQX_EPI_ACT | VQX_EPI_ACT2 |
                         VQX_EPI_OUTF32;
__host__ __device__ constexpr int ek_mask(int ek) {
  return ek == EK_NONE ? VQX_EPI_OUTF32
       : ek == EK_ELEM ? kEpiElem
       : ek == EK_GNADD ? kEpiElem | VQX_EPI_GNADD
       : ek == EK_SPLIT ? kEpiElem | VQX_EPI_SPLIT
       : ek == EK_COLSUM ? kEpiElem | VQX_EPI_COLSUM
       : ek == EK_GNSTATS ? kEpiElem | VQX_EPI_GNSTATS
       : ek == EK_GNBWD ? kEpiElem | VQX_EPI_COLSUM | VQX_EPI_GNBWD
       : ~0;
}

// Row operands of a bf16 fused epilogue, prefetched into registers for the
// thread's 8 (slab, pass) rows right after the prologue DMA is issued
// (conv_gemm_kernel, FWD), instead of one dependent load per row pass inside
// the epilogue.  Two slots per row; the roles are picked from the flags in
// the order GroupNorm input (GNADD / GNBWD), its second GLU half, mask,
// residual; operands without a slot are loaded in the epilogue as before.
// The 1x1 epilogues are bound by the burst of HBM traffic every workgroup
// issues at the same moment, not by these latencies: the prefetch buys 3-8%
// (tools/lab/k1_lab.cpp).
enum { EPR_NONE = 0, EPR_GNH, EPR_GNH2, EPR_MASK, EPR_RES };
typedef unsigned u32x4e_t __attribute__((ext_vector_type(4)));  // plain vector (HIP's uint4 is a union: kept in scratch)
struct EpiRows {
  u32x4e_t r0[8], r1[8];
  int k0, k1;
};

template <int EK, int I0 = 0, int NR = 8>  // slots I0 .. I0+NR-1 ((slab, pass) = (i >> 2, i & 3))
__device__ __forceinline__ void epi_prefetch(const GemmParams& P, int m0, int n0, int tid, EpiRows& R) {
  constexpr int EM = ek_mask(EK);
  const int epi = P.epi & EM;
  const int er = tid >> 4, col = n0 + (tid & 15) * 8;
  const bool to_out2 = (epi & VQX_EPI_SPLIT) && col >= P.split_col;  // neither mask nor res read there
  const bool g = epi & (VQX_EPI_GNADD | VQX_EPI_GNBWD), g2 = (epi & VQX_EPI_GNBWD) && P.gn_glu;  // g2 implies g
  const bool mk = (epi & VQX_EPI_MASK) && !to_out2, rs = (epi & VQX_EPI_RES) && !to_out2;
  const int k0 = g ? EPR_GNH : mk ? EPR_MASK : rs ? EPR_RES : EPR_NONE;
  const int k1 = g ? (g2 ? EPR_GNH2 : mk ? EPR_MASK : rs ? EPR_RES : EPR_NONE) : (mk && rs) ? EPR_RES : EPR_NONE;
  R.k0 = k0;
  R.k1 = k1;
  auto addr = [&](int k, int64_t row) -> const u32x4e_t* {
    const bf16_t* b = k == EPR_MASK ? (const bf16_t*)P.mask + row * P.ldmask
                    : k == EPR_RES  ? (const bf16_t*)P.res + row * P.ldres
                                    : (const bf16_t*)P.gn_h + row * P.ldgn + (k == EPR_GNH2 ? P.Nc : 0);
    return (const u32x4e_t*)(b + col);
  };
  static_for<NR>([&](auto i_c) __attribute__((always_inline)) {
    constexpr int i = I0 + decltype(i_c)::value;
    const int64_t row = (int64_t)m0 + (i >> 2) * 64 + (i & 3) * 16 + er;
    const bool ok = row < P.n_rows && col < P.Nc;
    const u32x4e_t z = {0u, 0u, 0u, 0u};
    R.r0[i] = (ok && k0 != EPR_NONE) ? *addr(k0, row) : z;
    R.r1[i] = (ok && k1 != EPR_NONE) ? *addr(k1, row) : z;
  });
}

__device__ __forceinline__ void unpack8(u32x4e_t u, float* f) {
  const unsigned w[4] = {u[0], u[1], u[2], u[3]};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[2 * k] = __uint_as_float(w[k] << 16);
    f[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}

// The prefetched operands of one epilogue row (by value: the 8-row arrays
// are indexed with compile-time pass numbers only, so they stay in VGPRs).
struct EpiOps {
  u32x4e_t p0, p1;
  int k0, k1;
};
template <int I, bool PRE>
__device__ __forceinline__ EpiOps epi_ops(const EpiRows* R) {
  EpiOps o = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, EPR_NONE, EPR_NONE};
  if constexpr (PRE) {  // (a runtime null test on R would keep the struct out of registers)
    o.p0 = R->r0[I];
    o.p1 = R->r1[I];
    o.k0 = R->k0;
    o.k1 = R->k1;
  }
  return o;
}

// Per-channel vectors of the thread's 8 output columns (bias, GroupNorm
// gamma/beta of both GLU halves), loaded once per tile instead of once per row
// pass when the epilogue prefetches (PRE).
struct EpiVec {
  float b[8], ga[8], be[8], gb[8], bb[8];
  float mr[4];  // GNBWD: the tile's utterance's (mean, rstd) pairs, valid when mr_ok
  bool mr_ok;
};
template <int EMASK>
__device__ __forceinline__ void epi_vec_load(const GemmParams& P, int col, EpiVec& V, int m0 = 0) {
  const int epi = P.epi & EMASK;
  V.mr_ok = false;
  if ((epi & VQX_EPI_GNBWD) && P.T % 128 == 0 && (P.gn_glu || P.gn_groups == 1)) {
    // every row of a 128-row tile lies in utterance m0 / T: one load per tile
    const int b = m0 / P.T, n = P.gn_glu ? 4 : 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) V.mr[i] = i < n ? P.gn_mr[b * n + i] : 0.f;
    V.mr_ok = true;
  }
  if (col >= P.Nc) return;
  if (epi & VQX_EPI_BIAS) ld8<float>(P.bias, col, V.b);
  if (epi & (VQX_EPI_GNADD | VQX_EPI_GNBWD)) {
    ld8<float>(P.gn_gamma, col, V.ga);
    if (!(epi & VQX_EPI_GNBWD) || P.gn_glu) ld8<float>(P.gn_beta, col, V.be);
    if ((epi & VQX_EPI_GNBWD) && P.gn_glu) {
      ld8<float>(P.gn_gamma, col + P.Nc, V.gb);
      ld8<float>(P.gn_beta, col + P.Nc, V.bb);
    }
  }
}
// 8 floats of a per-channel vector: the hoisted copy, else from memory
template <bool PRE>
__device__ __forceinline__ void vec8(const float (&pre)[8], const float* p, int64_t i, float* f) {
  if constexpr (PRE) {
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = pre[e];
  } else {
    ld8<float>(p, i, f);
  }
}

// 8 values of a row operand: from the prefetched slot holding `role`, else from memory
template <typename T>
__device__ __forceinline__ void row_op(const EpiOps& o, int role, const void* base, int64_t off, float* t) {
  if constexpr (sizeof(T) == 2) {
    if (o.k0 == role) { unpack8(o.p0, t); return; }
    if (o.k1 == role) { unpack8(o.p1, t); return; }
  }
  ld8<T>(base, off, t);
}

// FWD/DGRAD epilogue on 8 consecutive output channels of one frame, in the
// order bias, row bias, activation-derivative mask, split to out2 (returns),
// residual, GroupNorm-apply add, activation, store.  `o`: prefetched row
// operands (none: k0 = k1 = EPR_NONE).
template <typename T, int EMASK, bool PRE = false>
__device__ __forceinline__ void epilogue8(const GemmParams& P, int64_t row, int col, float* v, const float* gmr,
                                          const EpiOps& o, const EpiVec& V) {
  const int epi = P.epi & EMASK;
  const int bidx = (epi & (VQX_EPI_ROWBIAS | VQX_EPI_GNADD)) ? (int)row / P.T : 0;  // 32-bit: n_rows < 2^31 (host-checked)
  float t[8];
  if (epi & VQX_EPI_BIAS) {
    vec8<PRE>(V.b, P.bias, col, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += t[e];
  }
  if (epi & VQX_EPI_ROWBIAS) {
    ld8<float>(P.rowbias, (int64_t)bidx * P.Nc + col, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += t[e];
  }
  if (epi & VQX_EPI_MASK) {
    row_op<T>(o, EPR_MASK, P.mask, row * P.ldmask + col, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= (t[e] > 0.f ? 1.f : P.mask_slope) * P.mask_scale;
  }
  if ((epi & VQX_EPI_SPLIT) && col >= P.split_col) {  // split_col % 8 == 0
    float* o2 = P.out2 + row * P.ldo2 + (col - P.split_col);
    if (P.out2_acc) {
      ld8<float>(o2, 0, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += t[e];
    }
    st8<float>(o2, 0, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;  // not part of y: no column-sum contribution
    return;
  }
  if (epi & VQX_EPI_RES) {
    row_op<T>(o, EPR_RES, P.res, row * P.ldres + col, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += t[e];
  }
  if (epi & VQX_EPI_GNADD) {
    float ga[8], be[8];
    row_op<T>(o, EPR_GNH, P.gn_h, row * P.ldgn + col, t);
    vec8<PRE>(V.ga, P.gn_gamma, col, ga);
    vec8<PRE>(V.be, P.gn_beta, col, be);
    const float mean = gmr[2 * bidx], rstd = gmr[2 * bidx + 1];  // gmr: P.gn_mr or the in-launch merge
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += (t[e] - mean) * rstd * ga[e] + be[e];
  }
  if (epi & (VQX_EPI_ACT | VQX_EPI_ACT2)) {
#pragma unroll
    for (int e = 0; e < 8; ++e) t[e] = apply_pro(v[e], P.epi_act, 1.f);
    if (epi & VQX_EPI_ACT2) {
      st8<T>(P.y2, row * P.ldy2 + col, t);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = t[e];
    }
  }
  if (P.out_f32) st8_nt<float, false>(P.y, row * P.ldy + col, v);
  else st8_nt<T, false>(P.y, row * P.ldy + col, v);
}

// GNBWD: GroupNorm-backward sums of this output (the GN input's gradient dy)
// for 8 consecutive channels of one frame: s[0..1] = (sum g*dh, sum g*dh*xhat)
// of group a, s[2..3] of group b (GLU: u = [a | b], dh through
// tanh(h_a)*sigmoid(h_b), layers.py:240-242).  u, mean/rstd, gamma, beta are
// the forward GroupNorm's (gn_h, gn_mr, gn_gamma, gn_beta).
template <typename T, bool PRE = false>
__device__ __forceinline__ void gnbwd8(const GemmParams& P, int64_t row, int col, const float* dy, float* s,
                                       const EpiOps& o, const EpiVec& V) {
  const int b = (int)row / P.T;
  float ua[8], ga[8];
  row_op<T>(o, EPR_GNH, P.gn_h, row * P.ldgn + col, ua);
  vec8<PRE>(V.ga, P.gn_gamma, col, ga);
  const bool mr_pre = PRE && V.mr_ok;  // the tile's utterance's (mean, rstd), loaded once per tile
  if (!P.gn_glu) {
    const int grp = P.gn_groups == 1 ? 0 : col / (P.Nc / P.gn_groups);
    const float m = mr_pre ? V.mr[0] : P.gn_mr[(b * P.gn_groups + grp) * 2];
    const float r = mr_pre ? V.mr[1] : P.gn_mr[(b * P.gn_groups + grp) * 2 + 1];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float g = ga[e] * dy[e];
      s[0] += g;
      s[1] = fmaf(g, (ua[e] - m) * r, s[1]);
    }
    return;
  }
  const int half = P.Nc;
  float ub[8], gb[8], ba[8], bb[8];
  row_op<T>(o, EPR_GNH2, P.gn_h, row * P.ldgn + col + half, ub);
  vec8<PRE>(V.gb, P.gn_gamma, col + half, gb);
  vec8<PRE>(V.be, P.gn_beta, col, ba);
  vec8<PRE>(V.bb, P.gn_beta, col + half, bb);
  const float ma = mr_pre ? V.mr[0] : P.gn_mr[b * 4], ra = mr_pre ? V.mr[1] : P.gn_mr[b * 4 + 1];
  const float mb = mr_pre ? V.mr[2] : P.gn_mr[b * 4 + 2], rb = mr_pre ? V.mr[3] : P.gn_mr[b * 4 + 3];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float xa = (ua[e] - ma) * ra, xb = (ub[e] - mb) * rb;
    const float ta = ftanh<sizeof(T) == 2>(xa * ga[e] + ba[e]);
    const float sb = fsigmoid<sizeof(T) == 2>(xb * gb[e] + bb[e]);
    const float dga = ga[e] * (dy[e] * sb * (1.f - ta * ta));
    const float dgb = gb[e] * (dy[e] * ta * (sb * (1.f - sb)));
    s[0] += dga;
    s[1] = fmaf(dga, xa, s[1]);
    s[2] += dgb;
    s[3] = fmaf(dgb, xb, s[3]);
  }
}

// Fragment-level prologue (LDS-DMA staging cannot transform data in flight).
template <int PRO>
__device__ __forceinline__ bf16x8_t pro_frag(bf16x8_t f, float s) {
  if constexpr (PRO == VQX_PRO_NONE) {
    return f;
  } else {
    uint4 u = __builtin_bit_cast(uint4, f);
    u = pro_chunk<bf16_t, PRO>(u, s);
    return __builtin_bit_cast(bf16x8_t, u);
  }
}
template <int PRO>
__device__ __forceinline__ f32x4_t pro_frag(f32x4_t f, float s) {
  if constexpr (PRO == VQX_PRO_NONE) {
    return f;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = apply_pro(f[i], PRO, s);
    return f;
  }
}


// One 16-B-per-lane LDS-DMA (buffer_load_dwordx4 ... lds: 1 KiB per wave,
// lane-linear at the wave-uniform LDS address `lds`).  Issued as inline asm,
// not through __builtin_amdgcn_raw_ptr_buffer_load_lds: the compiler's
// waitcnt pass has no alias information for ds_read_b64_tr_b16, so after a
// builtin DMA it put `s_waitcnt vmcnt(0)` in front of the first transposed
// LDS read of every K-step -- the next stage's DMA landed before the current
// stage was multiplied, and DGRAD / WGRAD main loops (whose transposed
// operands use those reads) never overlapped staging with MFMAs.  Every
// kernel orders its DMAs explicitly (counted `s_waitcnt vmcnt` + s_barrier
// before a stage is read; the loops drain to vmcnt(0) before the epilogue
// reuses the staging LDS), so hiding them from the pass is safe; M0 (the
// DMA's LDS base) is set in the same statement.  An SALU write of M0 needs
// one wait state before an LDS-DMA reads it; the hazard recognizer that
// inserts it for the builtin does not look inside inline asm, hence the
// explicit s_nop.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, unsigned off) {
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(VQX_LDS(void)*)lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(la), "v"(off), "s"(r)
               : "memory", "m0");
}

// vmcnt immediate from a small runtime count (0..8, 10, 12, 16; anything else waits for all)
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// Epilogue of a 128x128 output tile (shared by conv_gemm_kernel and
// conv_tr_kernel).  The accumulator tile goes through LDS one 64-row slab at a
// time so the epilogue reads and writes whole rows: 16 lanes x 8 consecutive
// columns per row, every global access 16 B and each row segment contiguous.
// Lane holds (before the transpose) output row wm*64 + mi*32 + r32 and, per
// register group gq, columns wn*64 + ni*32 + 8*gq + 4*h + (0..3).  Needs
// 44 KiB of `smem`; the caller's staging buffers must be free.  `tid` is the
// thread's index in the 4-wave group that owns the tile (conv_tr8_kernel runs
// two such groups side by side; every group passes the same barriers).
template <typename T, int MODE, int EK, bool PRE = false, bool PREVEC = PRE>
__device__ __forceinline__ void tile_epilogue(const GemmParams& P, f32x16_t (&acc)[2][2], char* smem, int m0, int n0,
                                              int tn, int split, const float* gmr, int tid,
                                              const EpiRows* R = nullptr) {
  constexpr int EMASK = ek_mask(EK);
  constexpr int SUB = 1;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int r32 = lane & 31, h = lane >> 5;
  constexpr int EP_LD = kBN + 4;  // floats; +4 keeps the b128 writes conflict-free
  constexpr int EROWS = 16 * SUB;  // rows per pass
  float* ep = (float*)smem;                 // [64][EP_LD]
  // the GroupNorm / COLSUM reductions of a slab run after its row passes and
  // their barrier, when ep is dead until the next slab's writes (behind the
  // reductions' own closing barrier): they share its LDS
  float* csr = (float*)smem;                // [EROWS][kBN]
  const int er = tid >> 4, ec = (tid & 15) * 8;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // COLSUM accumulators
  float mn = 0.f, mm = 0.f, mq = 0.f;                       // GNSTATS running (count, mean, M2)
  float gs[4] = {0.f, 0.f, 0.f, 0.f};                       // GNBWD sums
  EpiVec V;
  if constexpr (PREVEC && MODE != MODE_WGRAD) epi_vec_load<EMASK>(P, n0 + ec, V, m0);
  __syncthreads();  // staging buffers are free
  // slab and pass are compile-time constants (static_for), so the prefetched
  // row operands R->r*[slab*4 + pass] are register-resident
  static_for<2 * SUB>([&](auto slab_c) __attribute__((always_inline)) {
    constexpr int slab = decltype(slab_c)::value;
    if (wm == slab) {
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            const f32x4_t v = {acc[mi][ni][4 * gq], acc[mi][ni][4 * gq + 1], acc[mi][ni][4 * gq + 2],
                               acc[mi][ni][4 * gq + 3]};
            *(f32x4_t*)(ep + (mi * 32 + r32) * EP_LD + wn * 64 + ni * 32 + 8 * gq + 4 * h) = v;
          }
    }
    __syncthreads();
    static_for<64 / EROWS>([&](auto pass_c) __attribute__((always_inline)) {
      constexpr int pass = decltype(pass_c)::value;
      const int lr = pass * EROWS + er;
      const f32x4_t lo = *(const f32x4_t*)(ep + lr * EP_LD + ec);
      const f32x4_t hi = *(const f32x4_t*)(ep + lr * EP_LD + ec + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      const int64_t row = (int64_t)m0 + slab * 64 + lr;
      const int col = n0 + ec;
      if constexpr (MODE == MODE_WGRAD) {
        if (row < P.Mc && col < P.Nc) {  // Nc % 8 == 0
          const int64_t at = (int64_t)split * P.Mc * P.Nc + row * P.Nc + col;
          if (sizeof(T) == 2 && P.slab_bf16) st8<bf16_t>(P.y, at, v);
          else st8_nt<float, false>((float*)P.y + at, 0, v);
        }
      } else {
        if (row < P.n_rows && col < P.Nc) {
          const EpiOps o = epi_ops<slab * 4 + pass, PRE>(R);
          epilogue8<T, EMASK, PREVEC>(P, row, col, v, gmr, o, V);
#pragma unroll
          for (int e = 0; e < 8; ++e) cs[e] += v[e];
          if (P.epi & EMASK & VQX_EPI_GNSTATS) {  // two-pass moments of the 8 values, merged
            float m8 = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) m8 += v[e];
            m8 *= 0.125f;
            float q8 = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) q8 = fmaf(v[e] - m8, v[e] - m8, q8);
            moments_merge(mn, mm, mq, 8.f, m8, q8);
          }
          if (P.epi & EMASK & VQX_EPI_GNBWD) gnbwd8<T, PREVEC>(P, row, col, v, gs, o, V);
        }
      }
    });
    __syncthreads();
    if constexpr (MODE != MODE_WGRAD) {
      // per-(128-row group, column tile) GroupNorm partials
      if ((P.epi & EMASK & (VQX_EPI_GNSTATS | VQX_EPI_GNBWD)) && (slab & 1)) {
        const int64_t grp_row = (int64_t)m0 + (slab >> 1) * 128;
        float* out = P.stat_part + ((grp_row / 128) * P.tiles_n + tn) * 4;
        if (P.epi & EMASK & VQX_EPI_GNSTATS) {
          // merge the 64 lanes of each wave, then the waves (deterministic order)
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            const float n2 = __shfl_xor(mn, o, 64), m2 = __shfl_xor(mm, o, 64), q2 = __shfl_xor(mq, o, 64);
            if ((lane & o) == 0) moments_merge(mn, mm, mq, n2, m2, q2);
            else { float a = n2, b = m2, c = q2; moments_merge(a, b, c, mn, mm, mq); mn = a; mm = b; mq = c; }
          }
          if (lane == 0) { csr[3 * wid] = mn; csr[3 * wid + 1] = mm; csr[3 * wid + 2] = mq; }
          __syncthreads();
          if (tid == 0 && grp_row < P.n_rows) {
            float a = csr[0], b = csr[1], c = csr[2];
            for (int w = 1; w < 4 * SUB; ++w) moments_merge(a, b, c, csr[3 * w], csr[3 * w + 1], csr[3 * w + 2]);
            out[0] = a; out[1] = b; out[2] = c; out[3] = 0.f;
          }
          mn = mm = mq = 0.f;
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float x = wave_sum(gs[k]);
            if (lane == 0) csr[4 * wid + k] = x;
            gs[k] = 0.f;
          }
          __syncthreads();
          if (tid < 4 && grp_row < P.n_rows) {
            float x = 0.f;
            for (int w = 0; w < 4 * SUB; ++w) x += csr[4 * w + tid];
            out[tid] = x;
          }
        }
        __syncthreads();
      }
      // per-128-row-group column sums of the stored values (bias gradient of
      // the layer this output feeds), reduced over the EROWS row lanes in LDS
      if ((P.epi & EMASK & VQX_EPI_COLSUM) && (slab & 1)) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          csr[er * kBN + ec + e] = cs[e];
          cs[e] = 0.f;
        }
        __syncthreads();
        const int64_t grp_row = (int64_t)m0 + (slab >> 1) * 128;
        if (tid < kBN && n0 + tid < P.Nc && grp_row < P.n_rows) {
          float t = 0.f;
#pragma unroll
          for (int r = 0; r < EROWS; ++r) t += csr[r * kBN + tid];
          P.colsum_part[(grp_row / 128) * P.Nc + n0 + tid] = t;
        }
        __syncthreads();
      }
    }
  });
}

// Staging layout.  The block tile is 128 x 128 with 4 waves in a 2 x 2 grid
// of 64 x 64 wave tiles.  A K-tile operand (A rows x BK, or BK x 128 B
// columns) is 128*BK*sizeof(T) bytes = PIECES pieces of 1 KiB; wave w fills
// pieces PW*w .. PW*w+PW-1 of each operand, lane l the 16-B chunk
// c = piece*64+l at LDS byte 16*c (lane-linear, as an LDS-DMA writes).  The
// XOR swizzle that keeps the fragment reads conflict-free is applied to the
// SOURCE chunk:
//   K-major,  RB-byte rows (RB = BK*sizeof(T)):  row = c / (RB/16),
//             data chunk = (c % (RB/16)) ^ kswz(row)
//   MN-major (256-B rows, bf16): row = c>>4, data chunk = (c&15) ^ mn_swz(row)
//   MN-major (512-B rows, f32):  row = c>>5, data chunk = c&31
// Operands go global -> LDS by buffer_load ... lds (no VGPR staging, no
// ds_write) through an NST-deep ring: NST-1 K-tiles are in flight while one
// is multiplied.  A counted vmcnt (this wave's pieces of the tiles still
// allowed in flight) retires tile kt+1 only, and a raw s_barrier publishes it
// and frees the buffer of tile kt for tile kt+NST.
//   BK=64, NST=2: 64 KiB per workgroup (the round-1 pipeline);
//   BK=32, NST=4: 64 KiB, three 16-KiB K-tiles in flight (bf16 default).
// Two 4-wave workgroups per CU either way.
// LDS bytes of conv_gemm_body: the NST-deep ring of A+B K-tiles (>= the epilogue's 44 KiB)
constexpr int kEpiBytes = 64 * (kBN + 4) * 4;  // tile_epilogue's LDS: one 64-row slab of the tile (33 KiB)
template <typename T, int BK, int NST>
__host__ __device__ constexpr int conv_gemm_smem() {
  return NST * 2 * 128 * BK * (int)sizeof(T) > kEpiBytes ? NST * 2 * 128 * BK * (int)sizeof(T) : kEpiBytes;
}

// The kernel body as a device function of (bid, nwg) = (this workgroup's
// index, workgroup count) of its own tile grid, on the caller's LDS, so that
// dual_*_kernel can host two GEMMs in one launch.
template <typename T, int MODE, int PRO, bool GEN, int BK, int NST, int EK>
__device__ __forceinline__ void conv_gemm_body(const GemmParams& P, int bid, int nwg, char* smem) {
  using C = Cfg<T>;
  constexpr int EPC = C::EPC, CPR = C::MNCPR, ES = sizeof(T);
  constexpr int BM = 128;
  constexpr int RB = BK * ES;                 // K-major row bytes (64 or 128)
  constexpr int KCH = RB / 16;                // 16-B chunks per K-major row
  constexpr int OP_BYTES = 128 * BK * ES;     // one operand's K-tile
  constexpr int PW = OP_BYTES / 1024 / 4;     // pieces per wave per operand
  constexpr int A_BYTES = OP_BYTES, STAGE = 2 * OP_BYTES;
  constexpr int NP = 2 * PW;                  // DMA pieces per wave per K-tile
  static_assert(conv_gemm_smem<T, BK, NST>() >= kEpiBytes, "epilogue staging needs 33 KiB of LDS");
  static_assert(BK % (16 / ES * 2) == 0 || ES == 4, "BK");
  static_assert(conv_gemm_smem<T, BK, NST>() >= NST * STAGE, "LDS");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int lin = xcd_remap(bid, nwg);
  const int tiles_mn = P.tiles_m * P.tiles_n;
  const int split = lin / tiles_mn;
  const int tmn = lin - split * tiles_mn;
  const int tm = tmn / P.tiles_n, tn = tmn - tm * P.tiles_n;
  const int m0 = tm * BM, n0 = tn * kBN;

  // GNADD with in-launch statistics (P.gn_tiles, T % 128 == 0: the tile is one
  // utterance b0): lane 0 of wave 0 merges the producing GEMM's tiles for b0
  // while the first K-tiles load (published by the main loop's barriers); the
  // first column tile of the utterance's first row tile stores them for the
  // backward.  gmr[2*bidx] then addresses gmr_s for bidx == b0.
  __shared__ float gmr_s[2];
  const float* gmr = P.gn_mr;
  if constexpr ((ek_mask(EK) & VQX_EPI_GNADD) != 0 && MODE == MODE_FWD) {
    if (P.gn_tiles != nullptr && (P.epi & VQX_EPI_GNADD)) {
      const int b0 = m0 / P.T;
      if (tid == 0) {
        const int rg = P.T / 128, ntn = P.Nc / 128;
        double n = 0.0, mean = 0.0, m2 = 0.0;
        for (int r = 0; r < rg; ++r)
          for (int t = 0; t < ntn; ++t) {
            const float* o = P.gn_tiles + ((int64_t)(b0 * rg + r) * ntn + t) * 4;
            const double nb = o[0];
            if (nb == 0.0) continue;
            const double d = (double)o[1] - mean;
            const double nn = n + nb;
            mean += d * nb / nn;
            m2 += (double)o[2] + d * d * n * nb / nn;
            n = nn;
          }
        const float var = n > 0.0 ? (float)(m2 / n) : 0.f;
        gmr_s[0] = (float)mean;
        gmr_s[1] = 1.0f / sqrtf(var + P.gn_eps);
        if (tn == 0 && m0 % P.T == 0) {
          ((float*)P.gn_mr)[2 * b0] = gmr_s[0];
          ((float*)P.gn_mr)[2 * b0 + 1] = gmr_s[1];
        }
      }
      gmr = gmr_s - 2 * b0;
    }
  }

  int64_t kbeg = 0, kend;
  if constexpr (MODE == MODE_WGRAD) {
    kbeg = (int64_t)split * P.k_per_split;
    kend = kbeg + P.k_per_split;
    if (kend > P.n_rows) kend = P.n_rows;
  } else {
    kend = P.K;
  }
  const int nk = (kend > kbeg) ? (int)((kend - kbeg + BK - 1) / BK) : 0;

  // ---------------- per-thread constant addressing
  unsigned aoff[PW], boff[PW];
  int amask[PW];      // FWD/DGRAD: bit j set <=> tap j keeps the frame inside its utterance
  int bsh[PW];        // WGRAD: krow + shift of the q chunk
  int ak[PW], bk[PW];  // k offset of the chunk inside the K-tile (elements / rows)
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int c = (PW * wid + i) * 64 + lane;
    amask[i] = 0;
    if constexpr (MODE != MODE_WGRAD) {
      const int row = c / KCH, kch = (c % KCH) ^ kswz<KCH>(row);
      const int64_t n = (int64_t)m0 + row;
      const int t = (int)(n % P.T);
      int msk = 0;
      if (n < P.n_rows)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int tt = t + j * P.dil - P.pad;
          msk |= (j < P.ntaps && tt >= 0 && tt < P.T) ? (1 << j) : 0;
        }
      amask[i] = msk;
      ak[i] = kch * EPC;
      aoff[i] = (unsigned)((n * P.lda + (GEN ? 0 : kch * EPC)) * ES);
    } else {
      const int krow = c / CPR;
      const int cch = (sizeof(T) == 2) ? ((c % CPR) ^ mn_swz(krow)) : (c % CPR);
      const int r = m0 + cch * EPC;
      ak[i] = krow;
      aoff[i] = r < P.Mc ? (unsigned)(((int64_t)krow * P.lda + r) * ES) : kOOB;
    }
  }
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int c = (PW * wid + i) * 64 + lane;
    bsh[i] = 0;
    if constexpr (MODE == MODE_FWD) {
      const int row = c / KCH, kch = (c % KCH) ^ kswz<KCH>(row);
      const int co = n0 + row;
      bk[i] = kch * EPC;
      boff[i] = co < P.Nc ? (unsigned)(((int64_t)co * P.K + kch * EPC) * ES) : kOOB;
    } else if constexpr (MODE == MODE_DGRAD) {
      const int krow = c / CPR;
      const int cch = (sizeof(T) == 2) ? ((c % CPR) ^ mn_swz(krow)) : (c % CPR);
      const int ci = n0 + cch * EPC;
      bk[i] = krow;
      boff[i] = ci < P.Nc ? (unsigned)(((int64_t)krow * P.ntaps * P.cdim + ci) * ES) : kOOB;
      if constexpr (GEN) boff[i] = ci < P.Nc ? (unsigned)(ci * ES) : kOOB;
    } else {
      const int krow = c / CPR;
      const int cch = (sizeof(T) == 2) ? ((c % CPR) ^ mn_swz(krow)) : (c % CPR);
      const int col = n0 + cch * EPC;
      const int j = tap_of(col, P.cdim, P.ntaps);
      const int cc = col - j * P.cdim;
      const int sh = P.sign * (j * P.dil - P.pad);
      bk[i] = krow;
      bsh[i] = krow + sh;
      // the q descriptor base sits (ntaps-1)*dil rows before the tile so shifted offsets stay >= 0
      boff[i] = col < P.Nc ? (unsigned)(((int64_t)(krow + sh + (P.ntaps - 1) * P.dil) * P.ldb + cc) * ES) : kOOB;
    }
  }

  // One buffer descriptor per operand for the whole kernel.  Its base sits
  // `lo` bytes before the operand (the largest negative im2col shift), so
  // every in-range offset is non-negative; per K-tile only a scalar byte
  // shift is added to each lane's offset (an out-of-range sentinel stays out
  // of range).
  int64_t a_lo = 0, b_lo = 0;
  if constexpr (MODE != MODE_WGRAD) a_lo = (int64_t)P.pad * P.lda * ES;
  if constexpr (MODE == MODE_WGRAD) b_lo = (int64_t)(P.ntaps - 1) * P.dil * P.ldb * ES;
  const __amdgpu_buffer_rsrc_t rsA = rsrc_at(P.a, -a_lo, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = rsrc_at(P.b, -b_lo, P.b_bytes);
  if constexpr (MODE != MODE_WGRAD) {
#pragma unroll
    for (int i = 0; i < PW; ++i) aoff[i] += (unsigned)a_lo;  // rebase to the descriptor
  }  // WGRAD: boff already carries the (ntaps-1)-row margin b_lo
  // incremental (tap, channel) position of the next K-tile to load (FWD/DGRAD fast path)
  int ld_tap = 0, ld_c0 = 0;
  int ld_t0 = MODE == MODE_WGRAD ? (int)(kbeg % P.T) : 0;  // WGRAD: frame-in-utterance of the next K-tile

  // Byte offsets of K-tile kt's chunks (kOOB where the im2col / edge reads zero).
  auto tile_offsets = [&](int kt, unsigned (&oa)[PW], unsigned (&ob)[PW]) {
    const int64_t k0 = kbeg + (int64_t)kt * BK;
    if constexpr (MODE != MODE_WGRAD) {
      if constexpr (!GEN) {
        const int tap = ld_tap, c0 = ld_c0;  // k0 == tap*kcin + c0
        ld_c0 += BK;
        if (ld_c0 >= P.kcin) { ld_c0 = 0; ld_tap += 1; }
        const unsigned ksa = (unsigned)(((tap * P.dil - P.pad) * P.lda + c0) * ES);
#pragma unroll
        for (int i = 0; i < PW; ++i) oa[i] = ((amask[i] >> tap) & 1) ? aoff[i] + ksa : kOOB;
        unsigned ksb;
        if constexpr (MODE == MODE_FWD) ksb = (unsigned)(k0 * ES);
        else  // forward weight We[co][j][ci] read as rows k = (j, co), taps flipped
          ksb = (unsigned)(((int64_t)c0 * P.ntaps * P.cdim + (int64_t)(P.ntaps - 1 - tap) * P.cdim) * ES);
#pragma unroll
        for (int i = 0; i < PW; ++i) ob[i] = boff[i] + ksb;
      } else {
#pragma unroll
        for (int i = 0; i < PW; ++i) {
          const int k = (int)k0 + ak[i];
          const int tap = tap_of(k, P.kcin, P.ntaps);
          const int ci = k - tap * P.kcin;
          const bool ok = k < P.K && ((amask[i] >> tap) & 1);
          oa[i] = ok ? aoff[i] + (unsigned)((((tap * P.dil - P.pad) * P.lda) + ci) * ES) : kOOB;
        }
        if constexpr (MODE == MODE_FWD) {
#pragma unroll
          for (int i = 0; i < PW; ++i) ob[i] = ((int)k0 + bk[i] < P.K) ? boff[i] + (unsigned)(k0 * ES) : kOOB;
        } else {
#pragma unroll
          for (int i = 0; i < PW; ++i) {
            const int k = (int)k0 + bk[i];
            const int j = tap_of(k, P.kcin, P.ntaps);
            const int co = k - j * P.kcin;
            ob[i] = (k < P.K && boff[i] != kOOB)
                        ? boff[i] + (unsigned)(((int64_t)co * P.ntaps * P.cdim + (P.ntaps - 1 - j) * P.cdim) * ES)
                        : kOOB;
          }
        }
      }
    } else {
      const unsigned ksa = (unsigned)(k0 * P.lda * ES);
      const unsigned ksb = (unsigned)(k0 * P.ldb * ES);
      // frame-in-utterance of the K-tile, advanced per call (tiles are loaded in
      // order; non-GEN: T % BK == 0) instead of a scalar 64-bit modulo per tile
      int t0 = ld_t0;
      if constexpr (!GEN) {
        ld_t0 += BK;
        if (ld_t0 >= P.T) ld_t0 -= P.T;
      } else {
        t0 = (int)((int)k0 % P.T);
      }
#pragma unroll
      for (int i = 0; i < PW; ++i) {
        unsigned offa = aoff[i] + ksa;
        if constexpr (GEN) {
          if (k0 + ak[i] >= kend) offa = kOOB;
        }
        oa[i] = offa;
      }
#pragma unroll
      for (int i = 0; i < PW; ++i) {
        int tt;
        if constexpr (!GEN) {
          tt = t0 + bsh[i];
        } else {
          const int64_t n = k0 + bk[i];
          tt = (int)(n % P.T) + (bsh[i] - bk[i]);
          if (n >= kend) tt = -1;
        }
        ob[i] = (tt >= 0 && tt < P.T) ? boff[i] + ksb : kOOB;
      }
    }
  };

  auto dma_tile = [&](int buf, int kt) {
    unsigned oa[PW], ob[PW];
    tile_offsets(kt, oa, ob);
    char* la = smem + buf * STAGE + wid * (PW * 1024);
    char* lb = smem + buf * STAGE + A_BYTES + wid * (PW * 1024);
#pragma unroll
    for (int i = 0; i < PW; ++i) dma16(rsA, la + i * 1024, oa[i]);
#pragma unroll
    for (int i = 0; i < PW; ++i) dma16(rsB, lb + i * 1024, ob[i]);
  };

  // LDS-DMA cannot transform data in flight: the prologue is applied to fragments after ds_read
  constexpr int FPRO_A = (MODE != MODE_WGRAD) ? PRO : VQX_PRO_NONE;
  constexpr int FPRO_B = (MODE == MODE_WGRAD) ? PRO : VQX_PRO_NONE;

  // acc[mi][ni]: mi = 32-block of the "row" operand (A tile), ni = of the B tile.
  // MFMA D = first(32 x k) * second(k x 32): first = B-tile fragment (contiguous
  // output index), second = A-tile fragment; D[row of first][col of second].
  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int r32 = lane & 31, h = lane >> 5;

  auto compute_tile = [&](int buf) {
    const char* la = smem + buf * STAGE;
    const char* lb = la + A_BYTES;
    const int acol = wm * 64;
    constexpr bool A_KMAJ = (MODE != MODE_WGRAD);
    constexpr bool B_KMAJ = (MODE == MODE_FWD);
    if constexpr (sizeof(T) == 2) {
      constexpr int KS = BK / 16;  // k-steps of v_mfma_f32_32x32x16_bf16
      const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
      typedef short s16x8_t __attribute__((ext_vector_type(8)));
      auto tr_frag = [&](const char* base, int colbase, int s) {
        const int kb = 16 * s + (g >> 1) * 8;
        const int ch = (colbase >> 3) + (p >> 1);
        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (VQX_LDS(s16x4_t)*)(base + mnmaj_off<T>(kb + q, ch) + 8 * (p & 1)));
        const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (VQX_LDS(s16x4_t)*)(base + mnmaj_off<T>(kb + 4 + q, ch) + 8 * (p & 1)));
        const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        return __builtin_bit_cast(bf16x8_t, v);
      };
      bf16x8_t af[KS][2], bfr[KS][2];
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          if constexpr (A_KMAJ) af[s][x] = *(const bf16x8_t*)(la + kmaj_off<KCH>(wm * 64 + x * 32 + r32, 2 * s + h));
          else af[s][x] = tr_frag(la, acol + x * 32 + (g & 1) * 16, s);
          if constexpr (B_KMAJ) bfr[s][x] = *(const bf16x8_t*)(lb + kmaj_off<KCH>(wn * 64 + x * 32 + r32, 2 * s + h));
          else bfr[s][x] = tr_frag(lb, wn * 64 + x * 32 + (g & 1) * 16, s);
        }
#pragma unroll
      for (int s = 0; s < KS; ++s) {
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          af[s][x] = pro_frag<FPRO_A>(af[s][x], P.pro_scale);
          bfr[s][x] = pro_frag<FPRO_B>(bfr[s][x], P.pro_scale);
        }
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[s][ni], af[s][mi], acc[mi][ni], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < BK / 8; ++s) {
        f32x4_t af[2], bfr[2];
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          if constexpr (A_KMAJ) {
            af[x] = *(const f32x4_t*)(la + kmaj_off<KCH>(wm * 64 + x * 32 + r32, 2 * s + h));
          } else {
            const int col = acol + x * 32 + r32;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) af[x][qq] = *(const float*)(la + (8 * s + 4 * h + qq) * 512 + col * 4);
          }
          if constexpr (B_KMAJ) {
            bfr[x] = *(const f32x4_t*)(lb + kmaj_off<KCH>(wn * 64 + x * 32 + r32, 2 * s + h));
          } else {
            const int col = wn * 64 + x * 32 + r32;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) bfr[x][qq] = *(const float*)(lb + (8 * s + 4 * h + qq) * 512 + col * 4);
          }
          af[x] = pro_frag<FPRO_A>(af[x], P.pro_scale);
          bfr[x] = pro_frag<FPRO_B>(bfr[x], P.pro_scale);
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(bfr[ni][qq], af[mi][qq], acc[mi][ni], 0, 0, 0);
      }
    }
  };

  // epilogue row operands of the bf16 FWD fused epilogues, prefetched with the
  // prologue (tools/lab/k1_lab.cpp, profiles/r02/k1_lab.txt: SPLIT 33.4 -> 30.6 us,
  // GNADD 26.9 -> 26.0 us; the DGRAD GNBWD epilogues, VALU-bound, ran 5-9% slower
  // with it and keep loading pass by pass)
  constexpr bool kPrefetch = sizeof(T) == 2 && EK != EK_NONE && EK != EK_ALL && MODE == MODE_FWD;
  // per-channel vectors (bias, GN affine) hoisted out of the row passes (FWD)
  constexpr bool kPreVec = kPrefetch;
  EpiRows rows;
  if constexpr (kPrefetch) {
    if (nk <= 0) epi_prefetch<EK>(P, m0, n0, tid, rows);
  }
  if (nk > 0) {
    // prologue: tiles 0 .. NST-2 in flight, then wait for tile 0
    const int pre = nk < NST - 1 ? nk : NST - 1;
#pragma unroll
    for (int t = 0; t < NST - 1; ++t)
      if (t < pre) dma_tile(t, t);
    if constexpr (kPrefetch) epi_prefetch<EK>(P, m0, n0, tid, rows);  // lands with the prologue DMA
    wait_vm(NP * (pre - 1));
    __builtin_amdgcn_s_barrier();
    int buf = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const int fbuf = (buf + NST - 1) % NST;  // buffer of tile kt+NST-1 == buffer of tile kt-1
      if (kt + NST - 1 < nk) dma_tile(fbuf, kt + NST - 1);
      compute_tile(buf);
      // tile kt+1 must have landed; tiles kt+2 .. min(nk, kt+NST)-1 may stay in flight
      if constexpr (NST == 2) {  // one tile in flight: it must have landed
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        int ahead = (kt + NST - 1 < nk ? kt + NST : nk) - (kt + 2);
        if (ahead < 0) ahead = 0;
        wait_vm(NP * ahead);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      buf = buf + 1 == NST ? 0 : buf + 1;
    }
  }

  tile_epilogue<T, MODE, EK, kPrefetch, kPreVec>(P, acc, smem, m0, n0, tn, split, gmr, (int)threadIdx.x, &rows);
}

template <typename T, int MODE, int PRO, bool GEN, int BK, int NST, int EK>
__global__ __launch_bounds__(256, 2) void conv_gemm_kernel(GemmParams P) {
  __shared__ __attribute__((aligned(16))) char smem[conv_gemm_smem<T, BK, NST>()];
  conv_gemm_body<T, MODE, PRO, GEN, BK, NST, EK>(P, blockIdx.x, gridDim.x, smem);
}

// Three workgroups per CU (48 KiB of LDS: 32-deep K-tiles in a 3-deep ring,
// <= 168 VGPRs) for 1x1 layers whose tile count lies between one and 1.5
// rounds of the two-per-CU kernel (config 2: the decoder's 512 -> 640
// res/skip conv, 640 tiles, which ran as a full round plus a quarter round).
// The 1x1 pipeline shape of the many-workgroups kernels (conv_gemm3_kernel,
// dual_k1_3_kernel): K-tile depth, ring depth and workgroups per CU.  Lab
// builds override them (build.py -D) for same-box A/Bs through VQX_LIB.
#ifndef VQX_K1_BK
#define VQX_K1_BK 32
#endif
#ifndef VQX_K1_NST
#define VQX_K1_NST 3
#endif
#ifndef VQX_K1_OCC
#define VQX_K1_OCC 3
#endif
template <typename T, int MODE, int PRO, bool GEN, int EK>
__global__ __launch_bounds__(256, VQX_K1_OCC) void conv_gemm3_kernel(GemmParams P) {
  __shared__ __attribute__((aligned(16))) char smem[conv_gemm_smem<T, VQX_K1_BK, VQX_K1_NST>()];
  conv_gemm_body<T, MODE, PRO, GEN, VQX_K1_BK, VQX_K1_NST, EK>(P, blockIdx.x, gridDim.x, smem);
}


// ---------------------------------------------------------------------------
// Tap-reuse conv GEMM: FWD / DGRAD of a 3-tap, pad-1 conv in bf16 when every
// 128-frame tile lies inside one utterance (T % 128 == 0).
//
// The implicit-im2col kernel above walks K = (tap, channel) and stages the
// activation tile once per tap, i.e. the same frames three times, shifted by
// one row.  Its main loop is bound by the L2 -> LDS staging rate
// (profiles/r01/gemm_lab.txt: operand staging alone takes 47 of 66 us on
// dec_in FWD).  Here a stage holds 32 channels of the 130 frames
// m0-1 .. m0+128 and the matching 32-channel slices of all three taps' weights
// (33 KiB), and the three taps are multiplied out of it by reading the
// activation fragments one or two rows further down: 1.5x the MFMA work per
// stage for 1.03x the staged bytes of a 64-deep K-tile, i.e. 0.69x the staged
// bytes per FLOP.
//
// Frame m0-1 (m0+128) is staged as zero when the tile starts (ends) an
// utterance: those rows are read only by tap 0 of the first row (tap 2 of the
// last row), which is exactly the im2col zero padding.  The row-shifted
// fragment reads stay conflict-free because the K-major swizzle depends on
// row % 16 only and a fragment's 16-lane groups cover 16 distinct residues.
// KSWZ for 32-B K-major rows (BKC = 16): rows r and r+8 share banks, so the
// 16-B half is flipped on bit 3 of the row; any 16 consecutive rows are then
// conflict-free for ds_read_b128, whatever the tap shift.
template <int KCH_>
__device__ __forceinline__ int tr_kswz(int row) {
  if constexpr (KCH_ == 2) return (row >> 3) & 1;
  else return kswz<KCH_>(row);
}
template <int KCH_>
__device__ __forceinline__ int tr_kmaj_off(int row, int ch) { return row * (16 * KCH_) + 16 * (ch ^ tr_kswz<KCH_>(row)); }

// BKC = channels per stage: 32 (2-deep ring, 33 KiB stages) or 16 (4-deep
// ring of 17 KiB stages: the same LDS, twice the prefetch distance)
// LDS bytes of conv_tr_body (the stage ring, at least the epilogue's 44 KiB)
template <int BKC>
__host__ __device__ constexpr int conv_tr_smem() {
  return (BKC == 32 ? 2 : 4) * (((130 * BKC * 2 + 1023) / 1024) * 1024 + 3 * 128 * BKC * 2) > 45056
             ? (BKC == 32 ? 2 : 4) * (((130 * BKC * 2 + 1023) / 1024) * 1024 + 3 * 128 * BKC * 2)
             : 45056;
}

template <int MODE, int EK, int BKC>
__device__ __forceinline__ void conv_tr_body(const GemmParams& P, int bid, int nwg, char* smem) {
  using T = bf16_t;
  constexpr int ES = 2, EPC = 8, KCH = BKC * ES / 16;  // 16-B chunks per K-major row
  constexpr int NST = BKC == 32 ? 2 : 4;
  constexpr int A_PIECES = (130 * BKC * ES + 1023) / 1024;  // 130 rows, rounded up to 1-KiB pieces
  constexpr int A_BYTES = A_PIECES * 1024;
  constexpr int TAP_BYTES = 128 * BKC * ES;            // one tap's weight slice
  constexpr int STAGE = A_BYTES + 3 * TAP_BYTES;
  constexpr int PWB = 3 * TAP_BYTES / 1024 / 4;        // weight pieces per wave per stage
  constexpr int TAP_PIECES = TAP_BYTES / 1024;
  static_assert(conv_tr_smem<BKC>() >= NST * STAGE && conv_tr_smem<BKC>() >= 45056, "LDS");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int lin = xcd_remap(bid, nwg);
  const int tm = lin / P.tiles_n, tn = lin - tm * P.tiles_n;
  const int m0 = tm * 128, n0 = tn * kBN;
  const int nk = P.kcin / BKC;

  // activation pieces of this wave: wid, wid+4, wid+8; stage row sr holds frame m0-1+sr
  unsigned aoff[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int piece = wid + 4 * i;
    const int c = piece * 64 + lane;
    const int row = c / KCH, kch = (c % KCH) ^ tr_kswz<KCH>(row);
    bool ok = piece < A_PIECES && row < 130;
    if (row == 0 && m0 % P.T == 0) ok = false;
    if (row == 129 && (m0 + 128) % P.T == 0) ok = false;
    // the descriptor base sits one activation row before P.a, so frame m0-1+row is at (m0+row) rows
    aoff[i] = ok ? (unsigned)((((int64_t)m0 + row) * P.lda + kch * EPC) * ES) : kOOB;
  }
  const int npa = (wid < A_PIECES ? 1 : 0) + (wid + 4 < A_PIECES ? 1 : 0) + (wid + 8 < A_PIECES ? 1 : 0);
  const int npw = npa + PWB;  // DMA instructions of this wave per stage
  // weight pieces wid*PWB .. : piece pb is tap pb / TAP_PIECES, 1-KiB slice pb % TAP_PIECES of it
  unsigned boff[PWB];
#pragma unroll
  for (int i = 0; i < PWB; ++i) {
    const int pb = wid * PWB + i;
    const int tap = pb / TAP_PIECES, c = (pb % TAP_PIECES) * 64 + lane;
    if constexpr (MODE == MODE_FWD) {  // We[co][tap*kcin + ci], K-major rows of BKC channels
      const int row = c / KCH, kch = (c % KCH) ^ tr_kswz<KCH>(row);
      const int co = n0 + row;
      boff[i] = co < P.Nc ? (unsigned)(((int64_t)co * P.K + tap * P.kcin + kch * EPC) * ES) : kOOB;
    } else {  // forward weight We[co][j][ci] read as rows co of tap j = 2 - tap (taps flipped)
      const int krow = c / 16, cch = (c % 16) ^ mn_swz(krow);
      const int ci = n0 + cch * EPC;
      boff[i] = ci < P.Nc ? (unsigned)(((int64_t)krow * 3 * P.cdim + (2 - tap) * P.cdim + ci) * ES) : kOOB;
    }
  }
  const __amdgpu_buffer_rsrc_t rsA = rsrc_at(P.a, -(int64_t)P.lda * ES, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = rsrc_at(P.b, 0, P.b_bytes);

  auto dma_stage = [&](int buf, int kt) {
    const int c0 = kt * BKC;
    const unsigned ksa = (unsigned)(c0 * ES);
    const unsigned ksb = MODE == MODE_FWD ? (unsigned)(c0 * ES) : (unsigned)((int64_t)c0 * 3 * P.cdim * ES);
    char* st = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (wid + 4 * i < A_PIECES) dma16(rsA, st + (wid + 4 * i) * 1024, aoff[i] + ksa);
#pragma unroll
    for (int i = 0; i < PWB; ++i) dma16(rsB, st + A_BYTES + (wid * PWB + i) * 1024, boff[i] + ksb);
  };

  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int r32 = lane & 31, h = lane >> 5;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  typedef short s16x8_t __attribute__((ext_vector_type(8)));

  auto compute_stage = [&](int buf) {
    const char* la = smem + buf * STAGE;
#pragma unroll
    for (int tap = 0; tap < 3; ++tap) {
      const char* lb = la + A_BYTES + tap * TAP_BYTES;
      constexpr int KS = BKC / 16;
      bf16x8_t af[KS][2], bfr[KS][2];
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          af[s][x] = *(const bf16x8_t*)(la + tr_kmaj_off<KCH>(wm * 64 + x * 32 + r32 + tap, 2 * s + h));
          if constexpr (MODE == MODE_FWD) {
            bfr[s][x] = *(const bf16x8_t*)(lb + tr_kmaj_off<KCH>(wn * 64 + x * 32 + r32, 2 * s + h));
          } else {
            const int kb = 16 * s + (g >> 1) * 8;
            const int ch = ((wn * 64 + x * 32 + (g & 1) * 16) >> 3) + (p >> 1);
            const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (VQX_LDS(s16x4_t)*)(lb + mnmaj_off<T>(kb + q, ch) + 8 * (p & 1)));
            const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (VQX_LDS(s16x4_t)*)(lb + mnmaj_off<T>(kb + 4 + q, ch) + 8 * (p & 1)));
            const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            bfr[s][x] = __builtin_bit_cast(bf16x8_t, v);
          }
        }
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[s][ni], af[s][mi], acc[mi][ni], 0, 0, 0);
    }
  };

  if (nk > 0) {
    // NST-1 stages in flight ahead of the one being multiplied
    const int pre = nk < NST - 1 ? nk : NST - 1;
#pragma unroll
    for (int t = 0; t < NST - 1; ++t)
      if (t < pre) dma_stage(t, t);
    if constexpr (NST == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else wait_vm(npw * (pre - 1));
    __builtin_amdgcn_s_barrier();
    int buf = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + NST - 1 < nk) dma_stage(buf == 0 ? NST - 1 : buf - 1, kt + NST - 1);
      compute_stage(buf);
      if constexpr (NST == 2) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {  // stage kt+1 must have landed; later ones may stay in flight
        int ahead = (kt + NST - 1 < nk ? kt + NST : nk) - (kt + 2);
        if (ahead < 0) ahead = 0;
        wait_vm(npw * ahead);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      buf = buf + 1 == NST ? 0 : buf + 1;
    }
  }
  tile_epilogue<T, MODE, EK>(P, acc, smem, m0, n0, tn, 0, P.gn_mr, (int)threadIdx.x);
}

template <int MODE, int EK, int BKC>
__global__ __launch_bounds__(256, 2) void conv_tr_kernel(GemmParams P) {
  __shared__ __attribute__((aligned(16))) char smem[conv_tr_smem<BKC>()];
  conv_tr_body<MODE, EK, BKC>(P, blockIdx.x, gridDim.x, smem);
}

// ---------------------------------------------------------------------------
// Tall tap-reuse conv GEMM: the same 3-tap FWD / DGRAD as conv_tr_kernel, with
// 256*SEGS frames x 128 columns per 8-wave workgroup (one per CU), for
// T % 256 == 0.  conv_tr_kernel is bound by the L2 -> LDS staging rate
// (~65 GB/s per CU): a 128-frame tile stages 9 KiB of frames + 24 KiB of
// weights per 32-channel stage for 3.1 MFLOP (95 FLOP per staged byte).  The
// staged frames serve all three taps, so a taller tile pays for its frames
// once while the weight slice is amortised over more rows: SEGS = 2 stages
// 33 KiB of frames + 24 KiB of weights for 12.6 MFLOP (219 FLOP/B), which
// moves the bound from the staging rate to the MFMA rate.
//
// Frames are staged per 256-frame segment with its own halo rows (row 0 =
// frame f0-1, row 257 = frame f0+256, zero at utterance edges), so every
// segment lies inside one utterance.  The tile is 2*SEGS quadrants of
// 128 x 128; the two 4-wave groups own SEGS quadrants each, every wave a
// 64 x 64 block of each, laid out exactly as conv_tr_kernel's waves so that
// each group runs tile_epilogue on its quadrants in its own 44 KiB of LDS.
// BKC = channels per stage: 32 (2-deep ring) or 16 (4-deep ring, two stages
// in flight behind counted vmcnt waits: the same LDS, twice the prefetch distance).
template <int MODE, int EK, int SEGS, int BKC = 32, int NST_ = (BKC == 32 ? 2 : 4)>
__global__ __launch_bounds__(512, 1) void conv_tr8_kernel(GemmParams P) {
  using T = bf16_t;
  constexpr int ES = 2, EPC = 8, KCH = BKC * ES / 16;  // 16-B chunks per K-major row
  constexpr int NST = NST_;  // ring depth: NST-1 stages in flight behind the one multiplied
  constexpr int SROWS = 258;                         // staged frames per segment
  constexpr int AROWS = SEGS * SROWS;
  constexpr int A_PIECES = (AROWS * BKC * ES + 1023) / 1024;
  constexpr int A_BYTES = A_PIECES * 1024;
  constexpr int PWA = (A_PIECES + 7) / 8;            // activation pieces per wave (some waves one fewer)
  constexpr int TAP_BYTES = 128 * BKC * ES;
  constexpr int TAP_PIECES = TAP_BYTES / 1024;
  constexpr int B_PIECES = 3 * TAP_PIECES;
  constexpr int PWB = (B_PIECES + 7) / 8;            // weight pieces per wave (wid, wid+8, ...)
  constexpr int STAGE = A_BYTES + 3 * TAP_BYTES;
  constexpr int EPI_BYTES = 45056;                   // tile_epilogue's LDS per group
  constexpr int SMEM = NST * STAGE > 2 * EPI_BYTES ? NST * STAGE : 2 * EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2, wm = (wid >> 1) & 1, wn = wid & 1;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lin / P.tiles_n, tn = lin - tm * P.tiles_n;
  const int64_t m0 = (int64_t)tm * (256 * SEGS);
  const int n0 = tn * kBN;
  const int nk = P.kcin / BKC;

  // activation pieces wid, wid+8, ...: stage row sr = seg*258 + r holds frame m0 + seg*256 - 1 + r
  unsigned aoff[PWA];
#pragma unroll
  for (int i = 0; i < PWA; ++i) {
    const int piece = wid + 8 * i;
    const int c = piece * 64 + lane;
    const int sr = c / KCH, kch = (c % KCH) ^ tr_kswz<KCH>(sr);
    const int seg = sr / SROWS, r = sr - seg * SROWS;
    const int64_t f0 = m0 + (int64_t)seg * 256;
    bool ok = piece < A_PIECES && sr < AROWS;
    if (r == 0 && f0 % P.T == 0) ok = false;
    if (r == SROWS - 1 && (f0 + 256) % P.T == 0) ok = false;
    // the descriptor base sits one activation row before P.a: frame f0-1+r is at row f0+r
    aoff[i] = ok ? (unsigned)(((f0 + r) * P.lda + kch * EPC) * ES) : kOOB;
  }
  unsigned boff[PWB];
#pragma unroll
  for (int i = 0; i < PWB; ++i) {
    const int pb = wid + 8 * i;
    const int tap = pb / TAP_PIECES, c = (pb % TAP_PIECES) * 64 + lane;
    if constexpr (MODE == MODE_FWD) {  // We[co][tap*kcin + ci], K-major rows of BKC channels
      const int row = c / KCH, kch = (c % KCH) ^ tr_kswz<KCH>(row);
      const int co = n0 + row;
      boff[i] = (pb < B_PIECES && co < P.Nc) ? (unsigned)(((int64_t)co * P.K + tap * P.kcin + kch * EPC) * ES) : kOOB;
    } else {  // forward weight We[co][j][ci] read as rows co of tap j = 2 - tap (taps flipped)
      const int krow = c / 16, cch = (c % 16) ^ mn_swz(krow);
      const int ci = n0 + cch * EPC;
      boff[i] = (pb < B_PIECES && ci < P.Nc)
                    ? (unsigned)(((int64_t)krow * 3 * P.cdim + (2 - tap) * P.cdim + ci) * ES) : kOOB;
    }
  }
  // DMA instructions of this wave per stage (the counted vmcnt waits of the 4-deep ring)
  const int npw = (A_PIECES - wid + 7) / 8 + (B_PIECES - wid + 7) / 8;
  const __amdgpu_buffer_rsrc_t rsA = rsrc_at(P.a, -(int64_t)P.lda * ES, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = rsrc_at(P.b, 0, P.b_bytes);

  auto dma_stage = [&](int buf, int kt) {
    const int c0 = kt * BKC;
    const unsigned ksa = (unsigned)(c0 * ES);
    const unsigned ksb = MODE == MODE_FWD ? (unsigned)(c0 * ES) : (unsigned)((int64_t)c0 * 3 * P.cdim * ES);
    char* st = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < PWA; ++i)
      if (wid + 8 * i < A_PIECES) dma16(rsA, st + (wid + 8 * i) * 1024, aoff[i] + ksa);
#pragma unroll
    for (int i = 0; i < PWB; ++i)
      if (wid + 8 * i < B_PIECES) dma16(rsB, st + A_BYTES + (wid + 8 * i) * 1024, boff[i] + ksb);
  };

  f32x16_t acc[SEGS][2][2];
#pragma unroll
  for (int j = 0; j < SEGS; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][i][k][e] = 0.f;

  const int r32 = lane & 31, h = lane >> 5;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  typedef short s16x8_t __attribute__((ext_vector_type(8)));
  // stage row of this wave's first fragment row in quadrant j (tap 0)
  int qrow[SEGS];
#pragma unroll
  for (int j = 0; j < SEGS; ++j) {
    const int qd = grp * SEGS + j;  // 128-row quadrant of the tile
    qrow[j] = (qd >> 1) * SROWS + (qd & 1) * 128 + wm * 64 + r32;
  }

  // (software-pipelining the fragment reads one (tap, 16-channel) group ahead
  // measured 2-10% slower: tools/lab/tr_lab.cpp, profiles/r02/tr_lab.txt)
  auto compute_stage = [&](int buf) {
    const char* la = smem + buf * STAGE;
#pragma unroll
    for (int tap = 0; tap < 3; ++tap) {
      const char* lb = la + A_BYTES + tap * TAP_BYTES;
      constexpr int KS = BKC / 16;
      bf16x8_t af[KS][SEGS][2], bfr[KS][2];
#pragma unroll
      for (int s = 0; s < KS; ++s) {
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          if constexpr (MODE == MODE_FWD) {
            bfr[s][x] = *(const bf16x8_t*)(lb + tr_kmaj_off<KCH>(wn * 64 + x * 32 + r32, 2 * s + h));
          } else {
            const int kb = 16 * s + (g >> 1) * 8;
            const int ch = ((wn * 64 + x * 32 + (g & 1) * 16) >> 3) + (p >> 1);
            const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (VQX_LDS(s16x4_t)*)(lb + mnmaj_off<T>(kb + q, ch) + 8 * (p & 1)));
            const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (VQX_LDS(s16x4_t)*)(lb + mnmaj_off<T>(kb + 4 + q, ch) + 8 * (p & 1)));
            const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            bfr[s][x] = __builtin_bit_cast(bf16x8_t, v);
          }
#pragma unroll
          for (int j = 0; j < SEGS; ++j)
            af[s][j][x] = *(const bf16x8_t*)(la + tr_kmaj_off<KCH>(qrow[j] + x * 32 + tap, 2 * s + h));
        }
      }
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < SEGS; ++j)
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              acc[j][mi][ni] =
                  __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[s][ni], af[s][j][mi], acc[j][mi][ni], 0, 0, 0);
    }
  };

  if (nk > 0) {
    // NST-1 stages in flight ahead of the one being multiplied
    const int pre = nk < NST - 1 ? nk : NST - 1;
#pragma unroll
    for (int t = 0; t < NST - 1; ++t)
      if (t < pre) dma_stage(t, t);
    if constexpr (NST == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else wait_vm(npw * (pre - 1));
    __builtin_amdgcn_s_barrier();
    int buf = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + NST - 1 < nk) dma_stage(buf == 0 ? NST - 1 : buf - 1, kt + NST - 1);
      compute_stage(buf);
      if constexpr (NST == 2) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {  // stage kt+1 must have landed; later ones may stay in flight
        int ahead = (kt + NST - 1 < nk ? kt + NST : nk) - (kt + 2);
        if (ahead < 0) ahead = 0;
        wait_vm(npw * ahead);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      buf = buf + 1 == NST ? 0 : buf + 1;
    }
  }
#pragma unroll
  for (int j = 0; j < SEGS; ++j)
    tile_epilogue<T, MODE, EK>(P, acc[j], smem + grp * EPI_BYTES, (int)(m0 + (grp * SEGS + j) * 128), n0, tn, 0,
                               P.gn_mr, tid & 255);
}

// ---------------------------------------------------------------------------
// Tap-reuse weight gradient of a 3-tap, pad-1 conv (bf16, T % 64 == 0):
//   S[r][j*cd + c] = sum_n p[n][r] * q[n + sign*(j-1)][c],  j = 0, 1, 2.
// The implicit-im2col WGRAD tiles the output 128 x 128, so each of the three
// taps' column blocks stages the same q frames again, one row shifted.  Here a
// workgroup owns 128 rows r x (3 taps x 64 channels c): a stage holds 64
// frames of p (16 KiB) and the 66 frames k0-1 .. k0+64 of q for its 64
// channels (9 KiB), and the three taps read the q fragments 0, 1 or 2 rows
// down.  24 MFMAs per wave per stage for 25 KiB staged: 2x the FLOPs per
// staged byte of the 128 x 128 tile.  Split-K as before; each 64-frame K-tile
// lies inside one utterance, so the halo frames are zero exactly when the
// K-tile starts (ends) an utterance.
//
// LDS: p as 256-B rows (mn_swz, read with ds_read_b64_tr_b16 like the other
// WGRAD), q as 128-B rows with the chunk XOR ((row >> 1) & 1) << 2: any four
// consecutive rows land in four distinct 64-B bank groups, whatever the tap
// shift.
__device__ __forceinline__ int q_off128(int row, int ch) { return row * 128 + 16 * (ch ^ (((row >> 1) & 1) << 2)); }

// In-launch ordered split-K reduction of one weight-gradient tile (ABI 127,
// vqx_wgrad_args.fixup_dw).  Every split has stored its bf16 partial of the
// tile write-through (sc1); each storing wave waits for its stores, the
// workgroup barrier joins them, and one lane adds to the tile's agent-scope
// counter.  The split whose add returns splits-1 is the last: it reads every
// split's partial of the tile with sc1 loads (the hand-off of
// MI355X_MICROARCH.md "inter-workgroup visibility", table row 1: write-through
// 16-B stores, one counter add per storing workgroup, the last adder told by
// the value its add returned, the other waves loading after a barrier),
// sums them in fp32 in the order vqx_weight_norm_bwd would (acc = 0, acc +=
// split s in order, or its interleaved split groups for short rows), stores
// the fp32 gradient and resets the counter for the next call.  No workgroup
// waits for another, so the grid needs no co-residency.
constexpr int kCpolSc1 = 16;  // buffer cache policy bit sc1 (gfx950)
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4_t bf16x4_lo(const u32x4_t& u) {
  return f32x4_t{__uint_as_float(u[0] << 16), __uint_as_float(u[0] & 0xffff0000u), __uint_as_float(u[1] << 16),
                 __uint_as_float(u[1] & 0xffff0000u)};
}
__device__ __forceinline__ f32x4_t bf16x4_hi(const u32x4_t& u) {
  return f32x4_t{__uint_as_float(u[2] << 16), __uint_as_float(u[2] & 0xffff0000u), __uint_as_float(u[3] << 16),
                 __uint_as_float(u[3] & 0xffff0000u)};
}
__device__ __forceinline__ void wgrad_tile_fixup(const GemmParams& P, int tmn, int r0, int c0,
                                              __amdgpu_buffer_rsrc_t rsY, char* smem) {
  constexpr int NT = 256;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slab stores have left
  __syncthreads();                                   // ... and every other wave's
  int* flag = (int*)smem;
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(P.fix_cnt + tmn, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = (int)old;
  }
  __syncthreads();
  if (*flag != P.splits - 1) return;  // uniform per workgroup
  if (threadIdx.x == 0) __hip_atomic_store(P.fix_cnt + tmn, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int tid = threadIdx.x;
  const int64_t ss2 = (int64_t)P.Mc * P.Nc * 2;  // bytes per split
  const int S = P.splits;
  // vqx_weight_norm_bwd's summation order for a row of Nc columns: one
  // sequential sum over the splits when the row has >= 256 four-column groups,
  // else G = min(S, 256 / groups) interleaved split groups added in group order
  // (wn_bwd_kernel, 256-thread blocks: vqx_misc.hip kWnThreads)
  const int nx4 = P.Nc / 4;
  const int G = nx4 >= 256 ? 1 : (S < 256 / nx4 ? S : 256 / nx4);
  // chunk (j, pass): row r0 + pass*32 + tid/8, columns j*cdim + c0 + (tid%8)*8 .. +7
  // (the slab store's lane map); two chunks per round, all their splits' loads in flight
  for (int it = 0; it < 12; it += 2) {
    int64_t at[2];
    bool ok[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = it + u, j = c >> 2, pass = c & 3;
      const int r = r0 + pass * (NT / 8) + (tid >> 3), cc = c0 + (tid & 7) * 8;
      ok[u] = r < P.Mc && cc < P.cdim;
      at[u] = (int64_t)r * P.Nc + j * P.cdim + cc;
    }
    f32x4_t t0[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    f32x4_t t1[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    for (int gi = 0; gi < G; ++gi) {  // split group gi: splits gi, gi+G, ... in order
      f32x4_t a0[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      f32x4_t a1[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      for (int s0 = gi; s0 < S; s0 += 8 * G) {
        u32x4_t v[2][8];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (ok[u] && s0 + k * G < S)
              v[u][k] = __builtin_amdgcn_raw_buffer_load_b128(rsY, (int)(at[u] * 2), (int)((s0 + k * G) * ss2),
                                                              kCpolSc1);
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (ok[u] && s0 + k * G < S) {
              a0[u] += bf16x4_lo(v[u][k]);
              a1[u] += bf16x4_hi(v[u][k]);
            }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {  // G == 1: 0 + a == a exactly (a sum from +0 is never -0)
        t0[u] += a0[u];
        t1[u] += a1[u];
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (ok[u]) {
        float* o = P.fix_dw + at[u];
        *(f32x4_t*)o = t0[u];
        *(f32x4_t*)(o + 4) = t1[u];
      }
  }
}

// LDS bytes of wgrad_tr_body: two 25-KiB stages, at least the slab-store
// staging (128 x 68 floats)
__host__ __device__ constexpr int wgrad_tr_smem() { return 2 * 25600 > 128 * 68 * 4 ? 2 * 25600 : 128 * 68 * 4; }

template <int EK>
__device__ __forceinline__ void wgrad_tr_body(const GemmParams& P, int bid, int nwg, char* smem) {
  using T = bf16_t;
  constexpr int ES = 2, EPC = 8, BK = 64, NT = 256;
  constexpr int A_BYTES = BK * 256;              // p: 64 frames x 128 r
  constexpr int B_PIECES = 9;                    // q: 66 frames x 64 c (72-row capacity)
  constexpr int B_BYTES = B_PIECES * 1024;
  constexpr int STAGE = A_BYTES + B_BYTES;       // 25 KiB
  constexpr int NST = 2;
  constexpr int EP_LD = 64 + 4;                  // epilogue row pitch (floats)
  constexpr int SMEM = NST * STAGE > 128 * EP_LD * 4 ? NST * STAGE : 128 * EP_LD * 4;
  static_assert(wgrad_tr_smem() == SMEM, "LDS");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wl = wid;
  const int wm = wl >> 1, wn = wl & 1;
  const int lin = xcd_remap(bid, nwg);
  const int tiles_mn = P.tiles_m * P.tiles_n;
  const int split = lin / tiles_mn;
  const int tmn = lin - split * tiles_mn;
  const int tm = tmn / P.tiles_n, tn = tmn - tm * P.tiles_n;
  const int r0 = tm * 128, c0 = tn * 64;
  const int64_t kbeg = (int64_t)split * P.k_per_split;
  int64_t kend = kbeg + P.k_per_split;
  if (kend > P.n_rows) kend = P.n_rows;
  const int nk = kend > kbeg ? (int)((kend - kbeg) / BK) : 0;

  // p pieces wl*4 .. wl*4+3 (16 per stage)
  unsigned aoff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = (wl * 4 + i) * 64 + lane;
    const int krow = c / 16, cch = (c % 16) ^ mn_swz(krow);
    const int r = r0 + cch * EPC;
    aoff[i] = r < P.Mc ? (unsigned)(((int64_t)krow * P.lda + r) * ES) : kOOB;
  }
  // q pieces wl, wl+4 and (wave 0 of the group) 8; stage row sr holds frame k0-1+sr
  unsigned boff[3];
  int bedge[3];  // 1: the k0-1 halo row, 2: the k0+64 halo row
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int piece = wl + 4 * i;
    const int c = piece * 64 + lane;
    const int row = c / 8, ch = (c % 8) ^ (((row >> 1) & 1) << 2);
    const int cc = c0 + ch * EPC;
    bedge[i] = row == 0 ? 1 : (row == 65 ? 2 : 0);
    // descriptor base one q row before P.b: frame k0-1+row sits at (k0+row) rows
    boff[i] = (piece < B_PIECES && row < 66 && cc < P.cdim) ? (unsigned)(((int64_t)row * P.ldb + cc) * ES) : kOOB;
  }
  const __amdgpu_buffer_rsrc_t rsA = rsrc_at(P.a, 0, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = rsrc_at(P.b, -(int64_t)P.ldb * ES, P.b_bytes);
  char* gsm = smem;

  int ld_t0 = (int)(kbeg % P.T);  // frame-in-utterance of the next K-tile to load
  auto dma_stage = [&](int buf, int kt) {  // called for kt = 0, 1, ... in order
    const int64_t k0 = kbeg + (int64_t)kt * BK;
    const int t0 = ld_t0;
    ld_t0 += BK;  // BK <= T (T % 64 == 0)
    if (ld_t0 >= P.T) ld_t0 -= P.T;
    const int edge = (t0 == 0 ? 1 : 0) | (t0 + BK == P.T ? 2 : 0);  // halo rows outside the utterance
    const unsigned ksa = (unsigned)(k0 * P.lda * ES), ksb = (unsigned)(k0 * P.ldb * ES);
    char* st = gsm + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) dma16(rsA, st + (wl * 4 + i) * 1024, aoff[i] + ksa);
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (wl + 4 * i < B_PIECES)
        dma16(rsB, st + A_BYTES + (wl + 4 * i) * 1024, (bedge[i] & edge) ? kOOB : boff[i] + ksb);
  };

  f32x16_t acc[2][3];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int r32 = lane & 31, h = lane >> 5;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  typedef short s16x8_t __attribute__((ext_vector_type(8)));
  const int ro0 = 1 - P.sign, ro2 = 1 + P.sign;  // stage-row offset of taps 0 and 2 (tap 1: 1)

  auto compute_stage = [&](int buf) {
    const char* la = gsm + buf * STAGE;
    const char* lb = la + A_BYTES;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8_t af[2], bfr[3];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int kb = 16 * s + (g >> 1) * 8;
        const int ch = ((wm * 64 + x * 32 + (g & 1) * 16) >> 3) + (p >> 1);
        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (VQX_LDS(s16x4_t)*)(la + mnmaj_off<T>(kb + q, ch) + 8 * (p & 1)));
        const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (VQX_LDS(s16x4_t)*)(la + mnmaj_off<T>(kb + 4 + q, ch) + 8 * (p & 1)));
        const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[x] = __builtin_bit_cast(bf16x8_t, v);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int ro = j == 0 ? ro0 : (j == 1 ? 1 : ro2);
        const int kb = 16 * s + (g >> 1) * 8 + ro;
        const int ch = ((wn * 32 + (g & 1) * 16) >> 3) + (p >> 1);
        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (VQX_LDS(s16x4_t)*)(lb + q_off128(kb + q, ch) + 8 * (p & 1)));
        const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (VQX_LDS(s16x4_t)*)(lb + q_off128(kb + 4 + q, ch) + 8 * (p & 1)));
        const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(bf16x8_t, v);
      }
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          acc[mi][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[j], af[mi], acc[mi][j], 0, 0, 0);
    }
  };

  if (nk > 0) {
    dma_stage(0, 0);
    wait_vm(0);
    __builtin_amdgcn_s_barrier();
    int buf = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) dma_stage(buf ^ 1, kt + 1);
      compute_stage(buf);
      wait_vm(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      buf ^= 1;
    }
  }

  // slab store, one tap at a time through LDS: rows of 64 channels, 8 lanes x 8 floats each
  float* ep = (float*)smem;
  const int64_t slab0 = (int64_t)split * P.Mc * P.Nc;
  const __amdgpu_buffer_rsrc_t rsY =
      __builtin_amdgcn_make_buffer_rsrc(P.y, (short)0, (int)((int64_t)P.splits * P.Mc * P.Nc * 2), 0x00020000);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    __syncthreads();
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const f32x4_t v = {acc[mi][j][4 * gq], acc[mi][j][4 * gq + 1], acc[mi][j][4 * gq + 2], acc[mi][j][4 * gq + 3]};
        *(f32x4_t*)(ep + (wm * 64 + mi * 32 + r32) * EP_LD + wn * 32 + 8 * gq + 4 * h) = v;
      }
    __syncthreads();
#pragma unroll
    for (int pass = 0; pass < 128 / (NT / 8); ++pass) {
      const int lr = pass * (NT / 8) + (tid >> 3), lc = (tid & 7) * 8;
      const int r = r0 + lr, cc = c0 + lc;
      if (r < P.Mc && cc < P.cdim) {
        const f32x4_t lo = *(const f32x4_t*)(ep + lr * EP_LD + lc);
        const f32x4_t hi = *(const f32x4_t*)(ep + lr * EP_LD + lc + 4);
        const int64_t at = slab0 + (int64_t)r * P.Nc + j * P.cdim + cc;
        if (P.slab_bf16 && P.fix_dw) {  // write-through (sc1): the tile's last split reads it in this launch
          const u32x4_t u = {pack_bf16x2(lo[0], lo[1]), pack_bf16x2(lo[2], lo[3]), pack_bf16x2(hi[0], hi[1]),
                             pack_bf16x2(hi[2], hi[3])};
          __builtin_amdgcn_raw_buffer_store_b128(u, rsY, (int)(at * 2), 0, kCpolSc1);
        } else if (P.slab_bf16) {
          const float v8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          st8<bf16_t>(P.y, at, v8);
        } else {
          float* o = (float*)P.y + at;
          *(f32x4_t*)o = lo;
          *(f32x4_t*)(o + 4) = hi;
        }
      }
    }
  }
  if (P.fix_dw) wgrad_tile_fixup(P, tmn, r0, c0, rsY, smem);
}

template <int EK>
__global__ __launch_bounds__(256, 2) void wgrad_tr_kernel(GemmParams P) {
  __shared__ __attribute__((aligned(16))) char smem[wgrad_tr_smem()];
  wgrad_tr_body<EK>(P, blockIdx.x, gridDim.x, smem);
}

}  // namespace vqx
