// Conv1d / ConvTranspose1d (stride 1) as implicit-im2col GEMMs on gfx950 MFMA.
//
// One kernel template covers the three products of a conv layer:
//   FWD   Y[n][co]      = sum_{j,ci} pro(x[n+j-pad][ci]) * We[co][j][ci]
//   DGRAD Y[n][ci]      = sum_{j,co} dy[n+j-pad][co]     * We[co][k-1-j][ci]
//   WGRAD S[r][j*cd+c]  = sum_n      p[n][r]             * pro(q[n+s(j-pad)][c])
// Frames (n = b*T + t) are the long GEMM dimension: 16,384 at config 2.
//
// Workgroup: 256 threads, 128x128 output tile, 4 waves in 2x2, each wave a
// 64x64 sub-tile = 2x2 MFMA blocks of 32x32.  bf16: v_mfma_f32_32x32x16_bf16,
// BK = 64; f32 (parity mode): v_mfma_f32_32x32x2_f32, BK = 32, an exact fp32
// fmaf chain.
//
// Staging: global -> registers -> LDS, double-buffered LDS, one barrier per
// K-tile, next tile's loads in flight during the MFMAs.  Loads are raw buffer
// loads: an offset past the descriptor's range returns zeros, which is how
// the im2col zero padding at utterance edges, the ragged M/N edges and the
// K tail are produced without branches.  When a K-tile lies inside one tap
// (cin % BK == 0: every large layer) the tap shift and the channel offset are
// folded into the wave-uniform descriptor base, so the per-chunk VALU work is
// one select.  K-contiguous operands live K-major in LDS (ds_read_b128, XOR
// swizzle); K-strided operands (weights in DGRAD, both operands in WGRAD) are
// stored as they lie in memory and read with ds_read_b64_tr_b16 (bf16) or
// ds_read_b32 (f32).
//
// The MFMA's first operand is the one whose index is contiguous in the output
// (channels for FWD/DGRAD, j*cd+c for WGRAD), so each lane ends up holding 4
// consecutive output elements per register group: the epilogue does vector
// loads/stores (8 B bf16, 16 B f32) for bias, residual, masks and results.
#include <hip/hip_ext.h>
#include <stdlib.h>

#include <vector>

#include "vqx_common.h"

namespace vqx {

constexpr int kBN = 128;  // tile width; the height is 128*SUB (conv_gemm_kernel)
constexpr unsigned kOOB = 0x80000000u;  // buffer offset that is always out of range -> loads 0
enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

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
};

template <typename T> struct Cfg;
template <> struct Cfg<bf16_t> { static constexpr int BK = 64, EPC = 8, MNCPR = 16; };
template <> struct Cfg<float> { static constexpr int BK = 32, EPC = 4, MNCPR = 32; };

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
      w[i] = (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    float f[4] = {__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = apply_pro(f[i], PRO, s);
    return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
  }
}

__device__ __forceinline__ int tap_of(int k, int c) { return (k >= c) + (k >= 2 * c); }

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

// LDS byte offsets of a 16-B chunk.
__device__ __forceinline__ int kmaj_off(int row, int ch) { return row * 128 + 16 * (ch ^ ((row >> 1) & 7)); }
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
    u.x = (unsigned)f2bf(f[0]) | ((unsigned)f2bf(f[1]) << 16);
    u.y = (unsigned)f2bf(f[2]) | ((unsigned)f2bf(f[3]) << 16);
    u.z = (unsigned)f2bf(f[4]) | ((unsigned)f2bf(f[5]) << 16);
    u.w = (unsigned)f2bf(f[6]) | ((unsigned)f2bf(f[7]) << 16);
    *(uint4*)((bf16_t*)p + i) = u;
  } else {
    const f32x4_t a = {f[0], f[1], f[2], f[3]}, b = {f[4], f[5], f[6], f[7]};
    *(f32x4_t*)((float*)p + i) = a;
    *(f32x4_t*)((float*)p + i + 4) = b;
  }
}

// FWD/DGRAD epilogue on 8 consecutive output channels of one frame, in the
// order bias, row bias, activation-derivative mask, split to out2 (returns),
// residual, GroupNorm-apply add, activation, store.
template <typename T>
__device__ __forceinline__ void epilogue8(const GemmParams& P, int64_t row, int col, float* v) {
  const int epi = P.epi;
  const int bidx = (epi & (VQX_EPI_ROWBIAS | VQX_EPI_GNADD)) ? (int)(row / P.T) : 0;
  float t[8];
  if (epi & VQX_EPI_BIAS) {
    ld8<float>(P.bias, col, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += t[e];
  }
  if (epi & VQX_EPI_ROWBIAS) {
    ld8<float>(P.rowbias, (int64_t)bidx * P.Nc + col, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += t[e];
  }
  if (epi & VQX_EPI_MASK) {
    ld8<T>(P.mask, row * P.ldmask + col, t);
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
    ld8<T>(P.res, row * P.ldres + col, t);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += t[e];
  }
  if (epi & VQX_EPI_GNADD) {
    float ga[8], be[8];
    ld8<T>(P.gn_h, row * P.ldgn + col, t);
    ld8<float>(P.gn_gamma, col, ga);
    ld8<float>(P.gn_beta, col, be);
    const float mean = P.gn_mr[2 * bidx], rstd = P.gn_mr[2 * bidx + 1];
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
  if (P.out_f32) st8<float>(P.y, row * P.ldy + col, v);
  else st8<T>(P.y, row * P.ldy + col, v);
}

// GNBWD: GroupNorm-backward sums of this output (the GN input's gradient dy)
// for 8 consecutive channels of one frame: s[0..1] = (sum g*dh, sum g*dh*xhat)
// of group a, s[2..3] of group b (GLU: u = [a | b], dh through
// tanh(h_a)*sigmoid(h_b), layers.py:240-242).  u, mean/rstd, gamma, beta are
// the forward GroupNorm's (gn_h, gn_mr, gn_gamma, gn_beta).
template <typename T>
__device__ __forceinline__ void gnbwd8(const GemmParams& P, int64_t row, int col, const float* dy, float* s) {
  const int b = (int)(row / P.T);
  float ua[8], ga[8];
  ld8<T>(P.gn_h, row * P.ldgn + col, ua);
  ld8<float>(P.gn_gamma, col, ga);
  if (!P.gn_glu) {
    const int grp = P.gn_groups == 1 ? 0 : col / (P.Nc / P.gn_groups);
    const float m = P.gn_mr[(b * P.gn_groups + grp) * 2], r = P.gn_mr[(b * P.gn_groups + grp) * 2 + 1];
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
  ld8<T>(P.gn_h, row * P.ldgn + col + half, ub);
  ld8<float>(P.gn_gamma, col + half, gb);
  ld8<float>(P.gn_beta, col, ba);
  ld8<float>(P.gn_beta, col + half, bb);
  const float ma = P.gn_mr[b * 4], ra = P.gn_mr[b * 4 + 1], mb = P.gn_mr[b * 4 + 2], rb = P.gn_mr[b * 4 + 3];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float xa = (ua[e] - ma) * ra, xb = (ub[e] - mb) * rb;
    const float ta = ftanh(xa * ga[e] + ba[e]);
    const float sb = fsigmoid(xb * gb[e] + bb[e]);
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

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, unsigned off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (VQX_LDS(void)*)lds, 16, (int)off, 0, 0, 0);
}

// Staging layout (both paths).  The block tile is BM x 128 with BM = 128*SUB
// (SUB = 1: 4 waves, 2 workgroups per CU; SUB = 2: 8 waves, 1 per CU, 25%
// fewer operand bytes per FLOP).  Waves form a (2*SUB) x 2 grid of 64x64
// wave tiles.  A K-tile operand is made of 16-KiB sub-tiles (A: SUB of them,
// B: one), each 16 pieces of 1 KiB; wave w fills A pieces 4w..4w+3 and B
// pieces (4/SUB)w.., lane l the 16-B chunk c = piece*64+l at LDS byte 16*c
// (lane-linear, as an LDS-DMA writes).  The XOR swizzle that keeps the
// fragment reads conflict-free is applied to the SOURCE chunk:
//   K-major  (128-B rows):  row = c>>3, data chunk = (c&7) ^ ((row>>1)&7)
//   MN-major (256-B rows, bf16): row = c>>4, data chunk = (c&15) ^ mn_swz(row)
//   MN-major (512-B rows, f32):  row = c>>5, data chunk = c&31
// (an MN-major A tile is SUB such sub-tiles side by side, 128 columns each).
// DMA = true: operands go global -> LDS by buffer_load ... lds (no VGPR
// staging, no ds_write), one K-tile ahead, `vmcnt(0)` + barrier per tile.
// DMA = false: global -> VGPR (two register sets) -> ds_write_b128.
template <typename T, int MODE, int PRO, bool GEN, bool DMA, int SUB>
__global__ __launch_bounds__(256 * SUB, SUB == 1 ? 2 : 1) void conv_gemm_kernel(GemmParams P) {
  using C = Cfg<T>;
  constexpr int BK = C::BK, EPC = C::EPC, CPR = C::MNCPR, ES = sizeof(T);
  constexpr int BM = 128 * SUB, NB = 4 / SUB;  // NB: B chunks per thread
  constexpr int A_BYTES = 16384 * SUB, STAGE = A_BYTES + 16384;
  // LDS-DMA ring depth: 2 for the 2-workgroups-per-CU tile, 3 (two K-tiles in
  // flight across each barrier) for the 1-workgroup-per-CU 256-row tile
  constexpr int NST = (DMA && SUB == 2) ? 3 : 2;
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles_mn = P.tiles_m * P.tiles_n;
  const int split = lin / tiles_mn;
  const int tmn = lin - split * tiles_mn;
  const int tm = tmn / P.tiles_n, tn = tmn - tm * P.tiles_n;
  const int m0 = tm * BM, n0 = tn * kBN;

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
  unsigned aoff[4], boff[NB];
  int amask[4];      // FWD/DGRAD: bit j set <=> tap j keeps the frame inside its utterance
  int bsh[NB];       // WGRAD: krow + shift of the q chunk
  int ak[4], bk[NB];  // k offset of the chunk inside the K-tile (elements / rows)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = (4 * wid + i) * 64 + lane;
    amask[i] = 0;
    if constexpr (MODE != MODE_WGRAD) {
      const int row = c >> 3, kch = (c & 7) ^ ((row >> 1) & 7);
      const int64_t n = (int64_t)m0 + row;
      const int t = (int)(n % P.T);
      int msk = 0;
      if (n < P.n_rows)
#pragma unroll
        for (int j = 0; j < 3; ++j) msk |= ((t + j - P.pad >= 0) && (t + j - P.pad < P.T)) ? (1 << j) : 0;
      amask[i] = msk;
      ak[i] = kch * EPC;
      aoff[i] = (unsigned)((n * P.lda + (GEN ? 0 : kch * EPC)) * ES);
    } else {
      const int sub = c >> 10, cc = c & 1023;
      const int krow = cc / CPR;
      const int cch = (sizeof(T) == 2) ? ((cc % CPR) ^ mn_swz(krow)) : (cc % CPR);
      const int r = m0 + sub * 128 + cch * EPC;
      ak[i] = krow;
      aoff[i] = r < P.Mc ? (unsigned)(((int64_t)krow * P.lda + r) * ES) : kOOB;
    }
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int c = (NB * wid + i) * 64 + lane;
    bsh[i] = 0;
    if constexpr (MODE == MODE_FWD) {
      const int row = c >> 3, kch = (c & 7) ^ ((row >> 1) & 7);
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
      const int j = tap_of(col, P.cdim);
      const int cc = col - j * P.cdim;
      const int sh = P.sign * (j - P.pad);
      bk[i] = krow;
      bsh[i] = krow + sh;
      // the q descriptor base sits (ntaps-1) rows before the tile so shifted offsets stay >= 0
      boff[i] = col < P.Nc ? (unsigned)(((int64_t)(krow + sh + P.ntaps - 1) * P.ldb + cc) * ES) : kOOB;
    }
  }

  // One buffer descriptor per operand for the whole kernel.  Its base sits
  // `lo` bytes before the operand (the largest negative im2col shift), so
  // every in-range offset is non-negative; per K-tile only a scalar byte
  // shift is added to each lane's offset (an out-of-range sentinel stays out
  // of range).
  int64_t a_lo = 0, b_lo = 0;
  if constexpr (MODE != MODE_WGRAD) a_lo = (int64_t)P.pad * P.lda * ES;
  if constexpr (MODE == MODE_WGRAD) b_lo = (int64_t)(P.ntaps - 1) * P.ldb * ES;
  const __amdgpu_buffer_rsrc_t rsA = rsrc_at(P.a, -a_lo, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = rsrc_at(P.b, -b_lo, P.b_bytes);
  if constexpr (MODE != MODE_WGRAD) {
#pragma unroll
    for (int i = 0; i < 4; ++i) aoff[i] += (unsigned)a_lo;  // rebase to the descriptor
  }  // WGRAD: boff already carries the (ntaps-1)-row margin b_lo
  // incremental (tap, channel) position of the next K-tile to load (FWD/DGRAD fast path)
  int ld_tap = 0, ld_c0 = 0;

  // Byte offsets of K-tile kt's chunks (kOOB where the im2col / edge reads zero).
  auto tile_offsets = [&](int kt, unsigned (&oa)[4], unsigned (&ob)[NB]) {
    const int64_t k0 = kbeg + (int64_t)kt * BK;
    if constexpr (MODE != MODE_WGRAD) {
      if constexpr (!GEN) {
        const int tap = ld_tap, c0 = ld_c0;  // k0 == tap*kcin + c0
        ld_c0 += BK;
        if (ld_c0 >= P.kcin) { ld_c0 = 0; ld_tap += 1; }
        const unsigned ksa = (unsigned)(((tap - P.pad) * P.lda + c0) * ES);
#pragma unroll
        for (int i = 0; i < 4; ++i) oa[i] = ((amask[i] >> tap) & 1) ? aoff[i] + ksa : kOOB;
        unsigned ksb;
        if constexpr (MODE == MODE_FWD) ksb = (unsigned)(k0 * ES);
        else  // forward weight We[co][j][ci] read as rows k = (j, co), taps flipped
          ksb = (unsigned)(((int64_t)c0 * P.ntaps * P.cdim + (int64_t)(P.ntaps - 1 - tap) * P.cdim) * ES);
#pragma unroll
        for (int i = 0; i < NB; ++i) ob[i] = boff[i] + ksb;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = (int)k0 + ak[i];
          const int tap = tap_of(k, P.kcin);
          const int ci = k - tap * P.kcin;
          const bool ok = k < P.K && ((amask[i] >> tap) & 1);
          oa[i] = ok ? aoff[i] + (unsigned)((((tap - P.pad) * P.lda) + ci) * ES) : kOOB;
        }
        if constexpr (MODE == MODE_FWD) {
#pragma unroll
          for (int i = 0; i < NB; ++i) ob[i] = ((int)k0 + bk[i] < P.K) ? boff[i] + (unsigned)(k0 * ES) : kOOB;
        } else {
#pragma unroll
          for (int i = 0; i < NB; ++i) {
            const int k = (int)k0 + bk[i];
            const int j = tap_of(k, P.kcin);
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
      const int t0 = (int)((int)k0 % P.T);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        unsigned offa = aoff[i] + ksa;
        if constexpr (GEN) {
          if (k0 + ak[i] >= kend) offa = kOOB;
        }
        oa[i] = offa;
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
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
    unsigned oa[4], ob[NB];
    tile_offsets(kt, oa, ob);
    char* la = smem + buf * STAGE + wid * 4096;
    char* lb = smem + buf * STAGE + A_BYTES + wid * (NB * 1024);
#pragma unroll
    for (int i = 0; i < 4; ++i) dma16(rsA, la + i * 1024, oa[i]);
#pragma unroll
    for (int i = 0; i < NB; ++i) dma16(rsB, lb + i * 1024, ob[i]);
  };

  auto load_tile = [&](int kt, uint4 (&ra)[4], uint4 (&rb)[NB]) {
    unsigned oa[4], ob[NB];
    tile_offsets(kt, oa, ob);
#pragma unroll
    for (int i = 0; i < 4; ++i) ra[i] = bload(rsA, oa[i]);
#pragma unroll
    for (int i = 0; i < NB; ++i) rb[i] = bload(rsB, ob[i]);
  };

  // register path: prologue applied at the store, after the load has landed
  auto store_tile = [&](int buf, const uint4 (&ra)[4], const uint4 (&rb)[NB]) {
    char* la = smem + buf * STAGE + wid * 4096 + lane * 16;
    char* lb = smem + buf * STAGE + A_BYTES + wid * (NB * 1024) + lane * 16;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *(uint4*)(la + i * 1024) = (MODE != MODE_WGRAD) ? pro_chunk<T, PRO>(ra[i], P.pro_scale) : ra[i];
#pragma unroll
    for (int i = 0; i < NB; ++i)
      *(uint4*)(lb + i * 1024) = (MODE == MODE_WGRAD) ? pro_chunk<T, PRO>(rb[i], P.pro_scale) : rb[i];
  };

  // DMA path: the prologue is applied to fragments after ds_read
  constexpr int FPRO_A = (DMA && MODE != MODE_WGRAD) ? PRO : VQX_PRO_NONE;
  constexpr int FPRO_B = (DMA && MODE == MODE_WGRAD) ? PRO : VQX_PRO_NONE;

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
    // MN-major A: this wave's 64 columns live in sub-tile wm>>1 at column (wm&1)*64
    const char* la_sub = la + (wm >> 1) * 16384;
    const int acol = (wm & 1) * 64;
    constexpr bool A_KMAJ = (MODE != MODE_WGRAD);
    constexpr bool B_KMAJ = (MODE == MODE_FWD);
    if constexpr (sizeof(T) == 2) {
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
      // all 16 fragments of the K-tile are read up front (64 VGPRs), so each
      // MFMA waits only for its own operands (counted lgkmcnt), not for a
      // drain of the LDS queue before every k-step
      bf16x8_t af[4][2], bfr[4][2];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          if constexpr (A_KMAJ) af[s][x] = *(const bf16x8_t*)(la + kmaj_off(wm * 64 + x * 32 + r32, 2 * s + h));
          else af[s][x] = tr_frag(la_sub, acol + x * 32 + (g & 1) * 16, s);
          if constexpr (B_KMAJ) bfr[s][x] = *(const bf16x8_t*)(lb + kmaj_off(wn * 64 + x * 32 + r32, 2 * s + h));
          else bfr[s][x] = tr_frag(lb, wn * 64 + x * 32 + (g & 1) * 16, s);
        }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
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
      for (int s = 0; s < 4; ++s) {
        f32x4_t af[2], bfr[2];
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          if constexpr (A_KMAJ) {
            af[x] = *(const f32x4_t*)(la + kmaj_off(wm * 64 + x * 32 + r32, 2 * s + h));
          } else {
            const int col = acol + x * 32 + r32;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) af[x][qq] = *(const float*)(la_sub + (8 * s + 4 * h + qq) * 512 + col * 4);
          }
          if constexpr (B_KMAJ) {
            bfr[x] = *(const f32x4_t*)(lb + kmaj_off(wn * 64 + x * 32 + r32, 2 * s + h));
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

  if constexpr (DMA && NST == 2) {
    // Tile kt+1 streams into the other buffer while tile kt is multiplied;
    // __syncthreads() waits vmcnt(0) (the DMA is a pending LDS write) and
    // orders every wave's reads of buffer kt&1 before its next refill.
    if (nk > 0) {
      dma_tile(0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) dma_tile((kt + 1) & 1, kt + 1);
        compute_tile(kt & 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
  } else if constexpr (DMA) {
    // Three-buffer ring: tiles kt+1 and kt+2 are in flight while tile kt is
    // multiplied.  A counted vmcnt (this wave's DMA pieces of one tile) retires
    // tile kt+1 only, and a raw s_barrier (no __syncthreads: its fence would
    // drain every DMA) publishes it and frees buffer kt%3 for tile kt+3.
    constexpr int NP = 4 + NB;  // DMA pieces per wave per tile
    if (nk > 0) {
      dma_tile(0, 0);
      if (nk > 1) {
        dma_tile(1, 1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NP) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      int buf = 0;
      for (int kt = 0; kt < nk; ++kt) {
        const int nbuf = buf == 2 ? 0 : buf + 1;
        const int fbuf = nbuf == 2 ? 0 : nbuf + 1;  // (kt + 2) % 3
        if (kt + 2 < nk) dma_tile(fbuf, kt + 2);
        compute_tile(buf);
        if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NP) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        buf = nbuf;
      }
    }
  } else {
    uint4 ra0[4], rb0[NB], ra1[4], rb1[NB];
    // Two register sets give every tile's loads two compute phases to land:
    // tile t is issued during tile t-2's MFMAs and written to LDS after t-1's.
    if (nk > 0) {
      load_tile(0, ra0, rb0);
      store_tile(0, ra0, rb0);
      if (nk > 1) load_tile(1, ra1, rb1);
      __syncthreads();
      int kt = 0;
      for (; kt + 2 <= nk; kt += 2) {  // no early exit: keeps acc in place across the halves
        if (kt + 2 < nk) load_tile(kt + 2, ra0, rb0);
        compute_tile(0);
        store_tile(1, ra1, rb1);
        __syncthreads();
        if (kt + 3 < nk) load_tile(kt + 3, ra1, rb1);
        compute_tile(1);
        if (kt + 2 < nk) store_tile(0, ra0, rb0);
        __syncthreads();
      }
      if (kt < nk) compute_tile(0);  // odd tail, already in buffer 0
    }
  }

  // ---------------- epilogue
  // The accumulator tile goes through LDS one 64-row slab at a time so the
  // epilogue reads and writes whole rows: 16 lanes x 8 consecutive columns
  // per row, every global access 16 B and each row segment contiguous.
  // Lane holds (before the transpose) output row wm*64 + mi*32 + r32 and,
  // per register group gq, columns wn*64 + ni*32 + 8*gq + 4*h + (0..3).
  constexpr int EP_LD = kBN + 4;  // floats; +4 keeps the b128 writes conflict-free
  constexpr int EROWS = 16 * SUB;  // rows per pass
  float* ep = (float*)smem;                 // [64][EP_LD]
  float* csr = (float*)(smem + 36864);      // COLSUM reduction [EROWS][kBN]
  const int er = tid >> 4, ec = (tid & 15) * 8;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // COLSUM accumulators
  float mn = 0.f, mm = 0.f, mq = 0.f;                       // GNSTATS running (count, mean, M2)
  float gs[4] = {0.f, 0.f, 0.f, 0.f};                       // GNBWD sums
  __syncthreads();  // staging buffers are free
#pragma unroll
  for (int slab = 0; slab < 2 * SUB; ++slab) {
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
#pragma unroll
    for (int pass = 0; pass < 64 / EROWS; ++pass) {
      const int lr = pass * EROWS + er;
      const f32x4_t lo = *(const f32x4_t*)(ep + lr * EP_LD + ec);
      const f32x4_t hi = *(const f32x4_t*)(ep + lr * EP_LD + ec + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      const int64_t row = (int64_t)m0 + slab * 64 + lr;
      const int col = n0 + ec;
      if constexpr (MODE == MODE_WGRAD) {
        if (row < P.Mc && col < P.Nc) {  // Nc % 8 == 0
          float* out = (float*)P.y + (int64_t)split * P.Mc * P.Nc + row * P.Nc + col;
          st8<float>(out, 0, v);
        }
      } else {
        if (row < P.n_rows && col < P.Nc) {
          epilogue8<T>(P, row, col, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) cs[e] += v[e];
          if (P.epi & VQX_EPI_GNSTATS) {  // two-pass moments of the 8 values, merged
            float m8 = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) m8 += v[e];
            m8 *= 0.125f;
            float q8 = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) q8 = fmaf(v[e] - m8, v[e] - m8, q8);
            moments_merge(mn, mm, mq, 8.f, m8, q8);
          }
          if (P.epi & VQX_EPI_GNBWD) gnbwd8<T>(P, row, col, v, gs);
        }
      }
    }
    __syncthreads();
    if constexpr (MODE != MODE_WGRAD) {
      // per-(128-row group, column tile) GroupNorm partials
      if ((P.epi & (VQX_EPI_GNSTATS | VQX_EPI_GNBWD)) && (slab & 1)) {
        const int64_t grp_row = (int64_t)m0 + (slab >> 1) * 128;
        float* out = P.stat_part + ((grp_row / 128) * P.tiles_n + tn) * 4;
        if (P.epi & VQX_EPI_GNSTATS) {
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
      if ((P.epi & VQX_EPI_COLSUM) && (slab & 1)) {
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
  }
}

// ---------------- launch probe (bench.py's roofline leg)
// While enabled, every conv GEMM is launched with hipExtLaunchKernelGGL and a
// start/stop event pair that the runtime stamps on the kernel's own dispatch
// packet, so the measured duration is the kernel's (no extra queue packets
// between kernels).  Events come from a pool reused across probe sessions.
struct ProbeRec {
  hipEvent_t start, stop;
  int info[5];  // dtype, mode, prologue, gen, dma
  double flops;
};
static bool g_probe_on = false;
static std::vector<ProbeRec> g_probe;
static std::vector<std::pair<hipEvent_t, hipEvent_t>> g_event_pool;
static size_t g_probe_used = 0;

template <typename K>
static void launch_gemm(K kernel, int grid, int threads, hipStream_t s, const GemmParams& P, const int info[5],
                        double flops) {
  if (!g_probe_on) {
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(threads), 0, s, P);
    return;
  }
  if (g_probe_used == g_event_pool.size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
      hipLaunchKernelGGL(kernel, dim3(grid), dim3(threads), 0, s, P);
      return;
    }
    g_event_pool.emplace_back(a, b);
  }
  auto ev = g_event_pool[g_probe_used++];
  ProbeRec r;
  r.start = ev.first;
  r.stop = ev.second;
  for (int i = 0; i < 5; ++i) r.info[i] = info[i];
  r.flops = flops;
  g_probe.push_back(r);
  hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(threads), 0, s, ev.first, ev.second, 0, P);
}

template <typename T, int MODE, bool GEN, bool DMA, int SUB>
static void launch_pro(const GemmParams& P, int grid, hipStream_t s) {
  const double flops = MODE == MODE_WGRAD ? 2.0 * (double)P.n_rows * P.Mc * P.Nc
                                          : 2.0 * (double)P.n_rows * P.Nc * P.K;
  const int info[5] = {sizeof(T) == 2 ? VQX_BF16 : VQX_F32, MODE, P.pro, GEN ? 1 : 0, (DMA ? 1 : 0) | (SUB == 2 ? 2 : 0)};
  const int nt = 256 * SUB;
  switch (P.pro) {
    case VQX_PRO_NONE: launch_gemm(conv_gemm_kernel<T, MODE, VQX_PRO_NONE, GEN, DMA, SUB>, grid, nt, s, P, info, flops); break;
    case VQX_PRO_LRELU: launch_gemm(conv_gemm_kernel<T, MODE, VQX_PRO_LRELU, GEN, DMA, SUB>, grid, nt, s, P, info, flops); break;
    case VQX_PRO_RELU: launch_gemm(conv_gemm_kernel<T, MODE, VQX_PRO_RELU, GEN, DMA, SUB>, grid, nt, s, P, info, flops); break;
    default: launch_gemm(conv_gemm_kernel<T, MODE, VQX_PRO_SCALE_RELU, GEN, DMA, SUB>, grid, nt, s, P, info, flops); break;
  }
}

// Staging variant: LDS-DMA by default; VQX_GEMM_STAGING=reg selects the
// register-staged pipeline (kept for A/B measurement, 128-row tiles only).
static bool use_dma() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("VQX_GEMM_STAGING");
    v = (e && e[0] == 'r') ? 0 : 1;
  }
  return v == 1;
}

// Tile height: 128 rows (SUB = 1, two 4-wave workgroups per CU).  The
// 256-row tile (SUB = 2, one 8-wave workgroup per CU, 25% fewer operand
// bytes per FLOP) measured equal or up to 12% slower on every config-2 layer
// (profiles/r01), so the automatic policy keeps 128; vqx_set_gemm_tile(2) /
// VQX_GEMM_SUB=2 selects it for A/B runs.
static int g_tile_policy = -1;  // 0 auto, 1 / 2 forced (vqx_set_gemm_tile)
static int pick_sub(int64_t tiles256) {
  if (g_tile_policy < 0) {
    const char* e = getenv("VQX_GEMM_SUB");
    g_tile_policy = (e && (e[0] == '1' || e[0] == '2')) ? e[0] - '0' : 0;
  }
  if (g_tile_policy) return g_tile_policy;
  (void)tiles256;
  return 1;
}

template <typename T, int MODE>
static void launch_mode(GemmParams& P, int64_t rows, int extra_mult, bool gen, hipStream_t s) {
  // rows: extent of the tile-M dimension; extra_mult: split-K factor (WGRAD)
  const int64_t t256 = ((rows + 255) / 256) * P.tiles_n * extra_mult;
  const int sub = use_dma() ? pick_sub(t256) : 1;
  P.tiles_m = (int)((rows + 128 * sub - 1) / (128 * sub));
  const int grid = P.tiles_m * P.tiles_n * extra_mult;
  if (!use_dma()) {
    if (gen) launch_pro<T, MODE, true, false, 1>(P, grid, s);
    else launch_pro<T, MODE, false, false, 1>(P, grid, s);
  } else if (sub == 2) {
    if (gen) launch_pro<T, MODE, true, true, 2>(P, grid, s);
    else launch_pro<T, MODE, false, true, 2>(P, grid, s);
  } else {
    if (gen) launch_pro<T, MODE, true, true, 1>(P, grid, s);
    else launch_pro<T, MODE, false, true, 1>(P, grid, s);
  }
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static int conv_common(const vqx_conv_args* a, int mode, hipStream_t s) {
  if (!a) { set_error("vqx_conv: null args"); return -1; }
  if (a->dtype != VQX_F32 && a->dtype != VQX_BF16) { set_error("vqx_conv: bad dtype %d", a->dtype); return -1; }
  const int epc = a->dtype == VQX_BF16 ? 8 : 4;
  const int es = a->dtype == VQX_BF16 ? 2 : 4;
  const int bk = a->dtype == VQX_BF16 ? 64 : 32;
  if (a->ntaps < 1 || a->ntaps > 3 || a->pad < 0 || a->pad >= a->ntaps + 1) { set_error("vqx_conv: ntaps %d / pad %d", a->ntaps, a->pad); return -1; }
  if (a->n_rows <= 0 || a->T <= 0 || a->n_rows % a->T) { set_error("vqx_conv: n_rows %lld not a multiple of T %d", (long long)a->n_rows, a->T); return -1; }
  if (a->cin <= 0 || a->cout <= 0 || a->cin % epc || a->ldx % epc || a->cin > a->ldx) { set_error("vqx_conv: cin %d / ldx %d must be multiples of %d", a->cin, a->ldx, epc); return -1; }
  if (a->cout % 8 || a->ldy % 8) { set_error("vqx_conv: cout %d / ldy %d must be multiples of 8", a->cout, a->ldy); return -1; }
  if (mode == MODE_DGRAD && a->cout % epc) { set_error("vqx_conv_dgrad: cout %d must be a multiple of %d", a->cout, epc); return -1; }
  if (!aligned16(a->x) || !aligned16(a->w)) { set_error("vqx_conv: x/w must be 16-byte aligned"); return -1; }
  if (a->prologue < 0 || a->prologue > 3 || (mode == MODE_DGRAD && a->prologue)) { set_error("vqx_conv: bad prologue %d", a->prologue); return -1; }
  const int epi = a->epilogue;
  if ((epi & VQX_EPI_BIAS) && (!a->bias || !aligned16(a->bias))) { set_error("vqx_conv: BIAS needs a 16-B aligned bias"); return -1; }
  if ((epi & VQX_EPI_ROWBIAS) && (!a->rowbias || !aligned16(a->rowbias))) { set_error("vqx_conv: ROWBIAS needs an aligned rowbias"); return -1; }
  if ((epi & VQX_EPI_RES) && (!a->res || a->ldres % 8 || !aligned16(a->res))) { set_error("vqx_conv: RES operand"); return -1; }
  if ((epi & VQX_EPI_MASK) && (!a->mask || a->ldmask % 8 || !aligned16(a->mask))) { set_error("vqx_conv: MASK operand"); return -1; }
  if ((epi & VQX_EPI_GNADD) && !(a->gn_h && a->gn_mean_rstd && a->gn_gamma && a->gn_beta && a->ldgn % 8 == 0 && aligned16(a->gn_h) && aligned16(a->gn_gamma) && aligned16(a->gn_beta))) { set_error("vqx_conv: GNADD operands"); return -1; }
  if ((epi & VQX_EPI_SPLIT) && (!a->out2 || a->split_col % 8 || a->ldo2 % 4 || !aligned16(a->out2))) { set_error("vqx_conv: SPLIT operands"); return -1; }
  if ((epi & VQX_EPI_ACT2) && (!a->y2 || a->ldy2 % 8 || !aligned16(a->y2))) { set_error("vqx_conv: ACT2 needs a 16-B aligned y2 with ldy2 %% 8 == 0"); return -1; }
  if ((epi & (VQX_EPI_ACT | VQX_EPI_ACT2)) && a->epi_act != VQX_PRO_LRELU && a->epi_act != VQX_PRO_RELU) { set_error("vqx_conv: epi_act must be LRELU or RELU"); return -1; }
  if (epi & (VQX_EPI_GNSTATS | VQX_EPI_GNBWD)) {
    const int G = a->gn_groups;
    if ((epi & VQX_EPI_GNSTATS) && (epi & VQX_EPI_GNBWD)) { set_error("vqx_conv: GNSTATS and GNBWD are exclusive"); return -1; }
    if (!a->stat_part || a->T % 128 || G < 1 || (epi & VQX_EPI_GNADD)) { set_error("vqx_conv: GN partials need stat_part, T %% 128 == 0, no GNADD"); return -1; }
    if ((epi & VQX_EPI_GNSTATS) && (a->cout % G || (a->cout / G) % 128)) { set_error("vqx_conv: GNSTATS needs cout/G %% 128 == 0"); return -1; }
    if (epi & VQX_EPI_GNBWD) {
      if (!(a->gn_h && a->gn_mean_rstd && a->gn_gamma && aligned16(a->gn_h) && aligned16(a->gn_gamma) && a->ldgn % 8 == 0)) { set_error("vqx_conv: GNBWD operands"); return -1; }
      if (a->gn_glu && (G != 2 || !a->gn_beta || !aligned16(a->gn_beta))) { set_error("vqx_conv: GNBWD glu needs G=2 and beta"); return -1; }
      if (!a->gn_glu && (a->cout % G || (a->cout / G) % 128)) { set_error("vqx_conv: GNBWD needs cout/G %% 128 == 0"); return -1; }
    }
  }
  if ((epi & VQX_EPI_COLSUM) && !a->colsum_part) { set_error("vqx_conv: COLSUM needs colsum_part [ceil(n_rows/128)][cout]"); return -1; }
  if (!a->y || !aligned16(a->y)) { set_error("vqx_conv: y must be non-null and 16-byte aligned"); return -1; }

  GemmParams P = {};
  P.a = a->x; P.b = a->w;
  P.a_bytes = ((a->n_rows - 1) * (int64_t)a->ldx + a->cin) * es;
  P.n_rows = a->n_rows; P.T = a->T; P.lda = a->ldx;
  P.kcin = a->cin; P.K = a->ntaps * a->cin; P.Mc = (int)a->n_rows; P.Nc = a->cout;
  P.b_bytes = (int64_t)a->ntaps * a->cin * a->cout * es;  // packed weight, either orientation
  P.ntaps = a->ntaps; P.pad = a->pad; P.sign = 1;
  P.cdim = a->cout;
  P.pro = a->prologue; P.pro_scale = a->pro_scale;
  P.tiles_n = (a->cout + kBN - 1) / kBN; P.splits = 1;  // tiles_m: launch_mode (tile height)
  P.y = a->y; P.ldy = a->ldy; P.epi = epi; P.out_f32 = (epi & VQX_EPI_OUTF32) ? 1 : 0;
  P.bias = a->bias; P.rowbias = a->rowbias; P.res = a->res; P.ldres = a->ldres;
  P.mask = a->mask; P.ldmask = a->ldmask; P.mask_slope = a->mask_slope; P.mask_scale = a->mask_scale;
  P.gn_h = a->gn_h; P.ldgn = a->ldgn; P.gn_mr = a->gn_mean_rstd; P.gn_gamma = a->gn_gamma; P.gn_beta = a->gn_beta;
  P.out2 = a->out2; P.ldo2 = a->ldo2; P.split_col = a->split_col; P.out2_acc = a->out2_accumulate;
  P.y2 = a->y2; P.ldy2 = a->ldy2; P.epi_act = a->epi_act;
  P.colsum_part = a->colsum_part;
  P.stat_part = a->stat_part; P.gn_groups = a->gn_groups; P.gn_glu = a->gn_glu;
  if (P.a_bytes > 0x7fffffffLL || P.b_bytes > 0x7fffffffLL) { set_error("vqx_conv: operand larger than 2 GiB"); return -1; }
  const bool gen = (a->cin % bk) != 0;
  if (a->dtype == VQX_BF16) {
    if (mode == MODE_FWD) launch_mode<bf16_t, MODE_FWD>(P, a->n_rows, 1, gen, s);
    else launch_mode<bf16_t, MODE_DGRAD>(P, a->n_rows, 1, gen, s);
  } else {
    if (mode == MODE_FWD) launch_mode<float, MODE_FWD>(P, a->n_rows, 1, gen, s);
    else launch_mode<float, MODE_DGRAD>(P, a->n_rows, 1, gen, s);
  }
  return launch_status(mode == MODE_FWD ? "vqx_conv1d_fwd" : "vqx_conv1d_dgrad");
}

}  // namespace vqx

using namespace vqx;

extern "C" int vqx_conv1d_fwd(const vqx_conv_args* a, vqx_stream_t stream) {
  return conv_common(a, MODE_FWD, (hipStream_t)stream);
}

extern "C" int vqx_conv1d_dgrad(const vqx_conv_args* a, vqx_stream_t stream) {
  return conv_common(a, MODE_DGRAD, (hipStream_t)stream);
}

extern "C" int vqx_conv1d_wgrad(const vqx_wgrad_args* a, vqx_stream_t stream) {
  if (!a) { set_error("vqx_conv1d_wgrad: null args"); return -1; }
  if (a->dtype != VQX_F32 && a->dtype != VQX_BF16) { set_error("vqx_conv1d_wgrad: bad dtype"); return -1; }
  const int epc = a->dtype == VQX_BF16 ? 8 : 4;
  const int es = a->dtype == VQX_BF16 ? 2 : 4;
  const int BK = a->dtype == VQX_BF16 ? 64 : 32;
  if (a->ntaps < 1 || a->ntaps > 3) { set_error("vqx_conv1d_wgrad: ntaps %d", a->ntaps); return -1; }
  if (a->n_rows <= 0 || a->T <= 0 || a->n_rows % a->T) { set_error("vqx_conv1d_wgrad: bad n_rows/T"); return -1; }
  if (a->r_dim % epc || a->c_dim % epc || a->ldp % epc || a->ldq % epc || a->c_dim % 8) { set_error("vqx_conv1d_wgrad: dims must be multiples of %d (c_dim of 8)", epc); return -1; }
  if (a->splits < 1) { set_error("vqx_conv1d_wgrad: splits < 1"); return -1; }
  if (!aligned16(a->p) || !aligned16(a->q) || !a->slabs || !aligned16(a->slabs)) { set_error("vqx_conv1d_wgrad: bad pointers"); return -1; }
  if (a->shift_sign != 1 && a->shift_sign != -1) { set_error("vqx_conv1d_wgrad: shift_sign must be +-1"); return -1; }
  GemmParams P = {};
  P.a = a->p; P.b = a->q; P.n_rows = a->n_rows; P.T = a->T; P.lda = a->ldp; P.ldb = a->ldq;
  P.a_bytes = ((a->n_rows - 1) * (int64_t)a->ldp + a->r_dim) * es;
  P.b_bytes = ((a->n_rows - 1) * (int64_t)a->ldq + a->c_dim) * es;
  if (P.a_bytes > 0x7fffffffLL || P.b_bytes > 0x7fffffffLL) { set_error("vqx_conv1d_wgrad: operand larger than 2 GiB"); return -1; }
  P.Mc = a->r_dim; P.Nc = a->ntaps * a->c_dim; P.ntaps = a->ntaps; P.pad = a->pad; P.sign = a->shift_sign;
  P.cdim = a->c_dim; P.pro = a->q_prologue; P.pro_scale = a->pro_scale;
  P.tiles_n = (P.Nc + kBN - 1) / kBN; P.splits = a->splits;  // tiles_m: launch_mode
  int64_t kps = (a->n_rows + a->splits - 1) / a->splits;
  kps = (kps + BK - 1) / BK * BK;
  P.k_per_split = kps;
  P.y = a->slabs;
  const bool gen = (a->T % BK) != 0 || (a->n_rows % BK) != 0;
  hipStream_t s = (hipStream_t)stream;
  if (a->dtype == VQX_BF16) launch_mode<bf16_t, MODE_WGRAD>(P, P.Mc, P.splits, gen, s);
  else launch_mode<float, MODE_WGRAD>(P, P.Mc, P.splits, gen, s);
  return launch_status("vqx_conv1d_wgrad");
}

extern "C" int vqx_set_gemm_tile(int32_t policy) {
  if (policy < 0 || policy > 2) { set_error("vqx_set_gemm_tile: policy %d not in {0, 1, 2}", policy); return -1; }
  g_tile_policy = policy;
  return 0;
}

extern "C" int vqx_probe_enable(int32_t on) {
  g_probe_on = on != 0;  // pause / resume; the log is kept
  return 0;
}

extern "C" int vqx_probe_clear(void) {
  g_probe.clear();
  g_probe_used = 0;
  return 0;
}

extern "C" int vqx_probe_count(int64_t* n) {
  if (!n) { set_error("vqx_probe_count: null"); return -1; }
  *n = (int64_t)g_probe.size();
  return 0;
}

extern "C" int vqx_probe_read(int64_t i, int32_t* info5, double* flops, float* ms) {
  if (i < 0 || i >= (int64_t)g_probe.size() || !info5 || !flops || !ms) { set_error("vqx_probe_read: bad index %lld", (long long)i); return -1; }
  const ProbeRec& r = g_probe[i];
  for (int k = 0; k < 5; ++k) info5[k] = r.info[k];
  *flops = r.flops;
  const hipError_t e = hipEventElapsedTime(ms, r.start, r.stop);
  if (e != hipSuccess) { set_error("vqx_probe_read: %s", hipGetErrorString(e)); return -1; }
  return 0;
}
