// Conv1d / ConvTranspose1d (stride 1) as implicit-im2col GEMMs on gfx950 MFMA.
//
// One kernel template covers the three products of a conv layer:
//   FWD   C[n][co]       = sum_{j,ci} pro(x[n+j-pad][ci]) * We[co][j][ci]
//   DGRAD C[n][ci]       = sum_{j,co} dy[n+j-pad][co]     * We[co][k-1-j][ci]
//   WGRAD C[r][j*cd+c]   = sum_n      p[n][r]             * pro(q[n+s(j-pad)][c])
// C rows of FWD/DGRAD are frames (B*T), so every conv of the VQ-VAE step is a
// GEMM with a 16,384-long M dimension at config 2.
//
// Tile: 128x128 C tile per 256-thread workgroup, 4 waves in a 2x2 grid, each
// wave a 64x64 sub-tile = 2x2 MFMA blocks of 32x32.  bf16 operands use
// v_mfma_f32_32x32x16_bf16 (BK=64), f32 operands v_mfma_f32_32x32x2_f32
// (BK=32, exact fp32 fmaf chain: the parity mode).  Operands are staged
// global->registers->LDS (double-buffered LDS, one barrier per K-tile, the
// next tile's global loads in flight during the MFMAs), which lets the
// staging pass apply the im2col shift/zero-padding, the activation prologue
// (LeakyReLU/ReLU) and dtype-agnostic 16-B chunk moves.  Operands whose K
// dimension is contiguous in memory are stored K-major in LDS and read with
// ds_read_b128; operands whose K dimension is strided (the weight in DGRAD,
// both operands in WGRAD) are stored as they lie in memory and read with the
// gfx950 transposing LDS read ds_read_b64_tr_b16 (bf16) or ds_read_b32 (f32).
#include "vqx_common.h"

namespace vqx {

constexpr int kBM = 128, kBN = 128, kThreads = 256;
enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

struct GemmParams {
  const void* a;   // FWD/DGRAD: activation [N][lda]; WGRAD: p [N][lda]
  const void* b;   // FWD/DGRAD: packed We [cout_f][ntaps*cin_f]; WGRAD: q [N][ldb]
  int64_t n_rows;  // frames
  int T, lda, ldb;
  int kcin;        // FWD/DGRAD: channels per tap on the K side
  int K;           // FWD/DGRAD: ntaps*kcin
  int Mc, Nc;      // C dims
  int ntaps, pad, sign;
  int cdim;        // DGRAD: cin of the forward layer (= Nc); WGRAD: c_dim
  int pro;
  float pro_scale;
  int tiles_m, tiles_n, splits;
  int64_t k_per_split;  // WGRAD
  // epilogue
  void* y;
  int ldy, epi, dtype_out_f32;
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

// tap index of a K offset (ntaps <= 3)
__device__ __forceinline__ int tap_of(int k, int c) { return (k >= c) + (k >= 2 * c); }

// LDS byte offsets of a 16-B chunk.
__device__ __forceinline__ int kmaj_off(int row, int ch) { return row * 128 + 16 * (ch ^ ((row >> 1) & 7)); }
__device__ __forceinline__ int mn_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
template <typename T>
__device__ __forceinline__ int mnmaj_off(int row, int ch) {
  if constexpr (sizeof(T) == 2) return row * 256 + 16 * (ch ^ mn_swz(row));
  else return row * 512 + 16 * ch;
}

template <typename T, int MODE, int PRO>
__global__ __launch_bounds__(kThreads, 2) void conv_gemm_kernel(GemmParams P) {
  using C = Cfg<T>;
  constexpr int BK = C::BK, EPC = C::EPC, CPR = C::MNCPR;
  constexpr int TILE_BYTES = 16384;
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int nwg = gridDim.x;
  const int lin = xcd_remap(blockIdx.x, nwg);
  const int tiles_mn = P.tiles_m * P.tiles_n;
  const int split = lin / tiles_mn;
  const int tmn = lin - split * tiles_mn;
  const int tm = tmn / P.tiles_n, tn = tmn - tm * P.tiles_n;
  const int m0 = tm * kBM, n0 = tn * kBN;

  int64_t kbeg = 0, kend;
  if constexpr (MODE == MODE_WGRAD) {
    kbeg = (int64_t)split * P.k_per_split;
    kend = kbeg + P.k_per_split;
    if (kend > P.n_rows) kend = P.n_rows;
  } else {
    kend = P.K;
  }
  const int nk = (kend > kbeg) ? (int)((kend - kbeg + BK - 1) / BK) : 0;

  // Per-thread constant row info for the FWD/DGRAD activation operand.
  int64_t a_n[4];
  int a_t[4];
  if constexpr (MODE != MODE_WGRAD) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + kThreads * i;
      a_n[i] = (int64_t)m0 + (c >> 3);
      a_t[i] = (int)(a_n[i] % P.T);
    }
  }

  const char* A = (const char*)P.a;
  const char* B = (const char*)P.b;
  uint4 ra[4], rb[4];
  const uint4 zero4 = make_uint4(0, 0, 0, 0);

  auto load_tile = [&](int kt) {
    const int64_t k0 = kbeg + (int64_t)kt * BK;
    if constexpr (MODE != MODE_WGRAD) {
      // A: activation, K-major rows = C rows (frames)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = tid + kThreads * i;
        const int kch = c & 7;
        const int k = (int)k0 + kch * EPC;
        const int tap = tap_of(k, P.kcin);
        const int ci = k - tap * P.kcin;
        const int tt = a_t[i] + tap - P.pad;
        const bool ok = (a_n[i] < P.n_rows) && (k < P.K) && (tt >= 0) && (tt < P.T);
        uint4 u = zero4;
        if (ok) u = *(const uint4*)(A + ((a_n[i] + tap - P.pad) * (int64_t)P.lda + ci) * sizeof(T));
        ra[i] = pro_chunk<T, PRO>(u, P.pro_scale);
      }
      if constexpr (MODE == MODE_FWD) {
        // B: packed weight, K-major rows = output channels
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = tid + kThreads * i;
          const int row = c >> 3, kch = c & 7;
          const int co = n0 + row;
          const int k = (int)k0 + kch * EPC;
          uint4 u = zero4;
          if (co < P.Nc && k < P.K) u = *(const uint4*)(B + ((int64_t)co * P.K + k) * sizeof(T));
          rb[i] = u;
        }
      } else {
        // B: forward weight We[co][j][ci] read as [k=(j,co)][ci], taps flipped
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = tid + kThreads * i;
          const int krow = c / CPR, cch = c % CPR;
          const int k = (int)k0 + krow;
          const int j = tap_of(k, P.kcin);
          const int co = k - j * P.kcin;
          const int ci = n0 + cch * EPC;
          uint4 u = zero4;
          if (k < P.K && ci < P.Nc)
            u = *(const uint4*)(B + ((int64_t)co * (P.ntaps * P.cdim) + (P.ntaps - 1 - j) * P.cdim + ci) * sizeof(T));
          rb[i] = u;
        }
      }
    } else {
      const int t0 = (int)(k0 % P.T);
      const bool tfast = (P.T % BK) == 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = tid + kThreads * i;
        const int krow = c / CPR, cch = c % CPR;
        const int64_t n = k0 + krow;
        const int r = m0 + cch * EPC;
        uint4 u = zero4;
        if (n < kend && r < P.Mc) u = *(const uint4*)(A + (n * P.lda + r) * sizeof(T));
        ra[i] = u;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = tid + kThreads * i;
        const int krow = c / CPR, cch = c % CPR;
        const int64_t n = k0 + krow;
        const int col = n0 + cch * EPC;
        const int j = tap_of(col, P.cdim);
        const int cc = col - j * P.cdim;
        const int sh = P.sign * (j - P.pad);
        const int t = tfast ? t0 + krow : (int)(n % P.T);
        const int tt = t + sh;
        uint4 u = zero4;
        if (n < kend && col < P.Nc && tt >= 0 && tt < P.T)
          u = *(const uint4*)(B + ((n + sh) * P.ldb + cc) * sizeof(T));
        rb[i] = pro_chunk<T, PRO>(u, P.pro_scale);
      }
    }
  };

  auto store_tile = [&](int buf) {
    char* la = smem + buf * 2 * TILE_BYTES;
    char* lb = la + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + kThreads * i;
      if constexpr (MODE != MODE_WGRAD) {
        *(uint4*)(la + kmaj_off(c >> 3, c & 7)) = ra[i];
      } else {
        *(uint4*)(la + mnmaj_off<T>(c / CPR, c % CPR)) = ra[i];
      }
      if constexpr (MODE == MODE_FWD) {
        *(uint4*)(lb + kmaj_off(c >> 3, c & 7)) = rb[i];
      } else {
        *(uint4*)(lb + mnmaj_off<T>(c / CPR, c % CPR)) = rb[i];
      }
    }
  };

  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int r32 = lane & 31, h = lane >> 5;

  auto compute_tile = [&](int buf) {
    const char* la = smem + buf * 2 * TILE_BYTES;
    const char* lb = la + TILE_BYTES;
    constexpr bool A_KMAJ = (MODE != MODE_WGRAD);
    constexpr bool B_KMAJ = (MODE == MODE_FWD);
    if constexpr (sizeof(T) == 2) {
      const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8_t af[2], bfr[2];
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          if constexpr (A_KMAJ) {
            const int row = wm * 64 + x * 32 + r32;
            af[x] = *(const bf16x8_t*)(la + kmaj_off(row, 2 * s + h));
          } else {
            const int colbase = wm * 64 + x * 32 + (g & 1) * 16;
            const int kb = 16 * s + (g >> 1) * 8;
            const int r0 = kb + q, r1 = kb + 4 + q;
            const int ch = (colbase >> 3) + (p >> 1);
            s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (VQX_LDS(s16x4_t)*)(la + mnmaj_off<T>(r0, ch) + 8 * (p & 1)));
            s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (VQX_LDS(s16x4_t)*)(la + mnmaj_off<T>(r1, ch) + 8 * (p & 1)));
            typedef short s16x8_t __attribute__((ext_vector_type(8)));
            s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            af[x] = __builtin_bit_cast(bf16x8_t, v);
          }
          if constexpr (B_KMAJ) {
            const int row = wn * 64 + x * 32 + r32;
            bfr[x] = *(const bf16x8_t*)(lb + kmaj_off(row, 2 * s + h));
          } else {
            const int colbase = wn * 64 + x * 32 + (g & 1) * 16;
            const int kb = 16 * s + (g >> 1) * 8;
            const int r0 = kb + q, r1 = kb + 4 + q;
            const int ch = (colbase >> 3) + (p >> 1);
            s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (VQX_LDS(s16x4_t)*)(lb + mnmaj_off<T>(r0, ch) + 8 * (p & 1)));
            s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (VQX_LDS(s16x4_t)*)(lb + mnmaj_off<T>(r1, ch) + 8 * (p & 1)));
            typedef short s16x8_t __attribute__((ext_vector_type(8)));
            s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            bfr[x] = __builtin_bit_cast(bf16x8_t, v);
          }
        }
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        f32x4_t af[2], bfr[2];
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          if constexpr (A_KMAJ) {
            const int row = wm * 64 + x * 32 + r32;
            af[x] = *(const f32x4_t*)(la + kmaj_off(row, 2 * s + h));
          } else {
            const int col = wm * 64 + x * 32 + r32;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) af[x][qq] = *(const float*)(la + (8 * s + 4 * h + qq) * 512 + col * 4);
          }
          if constexpr (B_KMAJ) {
            const int row = wn * 64 + x * 32 + r32;
            bfr[x] = *(const f32x4_t*)(lb + kmaj_off(row, 2 * s + h));
          } else {
            const int col = wn * 64 + x * 32 + r32;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) bfr[x][qq] = *(const float*)(lb + (8 * s + 4 * h + qq) * 512 + col * 4);
          }
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[mi][qq], bfr[ni][qq], acc[mi][ni], 0, 0, 0);
      }
    }
  };

  if (nk > 0) {
    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = (kt + 1) < nk;
      if (more) load_tile(kt + 1);
      compute_tile(kt & 1);
      if (more) store_tile((kt + 1) & 1);
      __syncthreads();
    }
  }

  // ---------------- epilogue ----------------
  if constexpr (MODE == MODE_WGRAD) {
    float* out = (float*)P.y + (int64_t)split * P.Mc * P.Nc;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int col = n0 + wn * 64 + ni * 32 + r32;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = m0 + wm * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
          if (row < P.Mc && col < P.Nc) out[(int64_t)row * P.Nc + col] = acc[mi][ni][e];
        }
      }
  } else {
    const int epi = P.epi;
    const int odt = P.dtype_out_f32 ? VQX_F32 : (sizeof(T) == 2 ? VQX_BF16 : VQX_F32);
    constexpr int idt = sizeof(T) == 2 ? VQX_BF16 : VQX_F32;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int col = n0 + wn * 64 + ni * 32 + r32;
        if (col >= P.Nc) continue;
        float bcol = (epi & VQX_EPI_BIAS) ? P.bias[col] : 0.f;
        float gam = 0.f, bet = 0.f;
        if (epi & VQX_EPI_GNADD) { gam = P.gn_gamma[col]; bet = P.gn_beta[col]; }
        const bool to2 = (epi & VQX_EPI_SPLIT) && col >= P.split_col;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int64_t row = (int64_t)m0 + wm * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
          if (row >= P.n_rows) continue;
          float v = acc[mi][ni][e] + bcol;
          int bidx = 0;
          if (epi & (VQX_EPI_ROWBIAS | VQX_EPI_GNADD)) bidx = (int)(row / P.T);
          if (epi & VQX_EPI_ROWBIAS) v += P.rowbias[(int64_t)bidx * P.Nc + col];
          if (epi & VQX_EPI_MASK) {
            const float mv = ld_dt(P.mask, row * P.ldmask + col, idt);
            v *= (mv > 0.f ? 1.f : P.mask_slope) * P.mask_scale;
          }
          if (to2) {
            float* o2 = P.out2 + row * P.ldo2 + (col - P.split_col);
            *o2 = P.out2_acc ? (*o2 + v) : v;
            continue;
          }
          if (epi & VQX_EPI_RES) v += ld_dt(P.res, row * P.ldres + col, idt);
          if (epi & VQX_EPI_GNADD) {
            const float hv = ld_dt(P.gn_h, row * P.ldgn + col, idt);
            v += (hv - P.gn_mr[2 * bidx]) * P.gn_mr[2 * bidx + 1] * gam + bet;
          }
          st_dt(P.y, row * P.ldy + col, v, odt);
        }
      }
  }
}

template <typename T, int MODE>
static void launch_mode(const GemmParams& P, int grid, hipStream_t s) {
  switch (P.pro) {
    case VQX_PRO_NONE: hipLaunchKernelGGL((conv_gemm_kernel<T, MODE, VQX_PRO_NONE>), dim3(grid), dim3(kThreads), 0, s, P); break;
    case VQX_PRO_LRELU: hipLaunchKernelGGL((conv_gemm_kernel<T, MODE, VQX_PRO_LRELU>), dim3(grid), dim3(kThreads), 0, s, P); break;
    case VQX_PRO_RELU: hipLaunchKernelGGL((conv_gemm_kernel<T, MODE, VQX_PRO_RELU>), dim3(grid), dim3(kThreads), 0, s, P); break;
    default: hipLaunchKernelGGL((conv_gemm_kernel<T, MODE, VQX_PRO_SCALE_RELU>), dim3(grid), dim3(kThreads), 0, s, P); break;
  }
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static int conv_common(const vqx_conv_args* a, int mode, hipStream_t s) {
  if (!a) { set_error("vqx_conv: null args"); return -1; }
  const int epc = a->dtype == VQX_BF16 ? 8 : 4;
  if (a->dtype != VQX_F32 && a->dtype != VQX_BF16) { set_error("vqx_conv: bad dtype %d", a->dtype); return -1; }
  if (a->ntaps < 1 || a->ntaps > 3) { set_error("vqx_conv: ntaps %d not in [1,3]", a->ntaps); return -1; }
  if (a->n_rows <= 0 || a->T <= 0 || a->n_rows % a->T) { set_error("vqx_conv: n_rows %lld not a multiple of T %d", (long long)a->n_rows, a->T); return -1; }
  if (a->cin <= 0 || a->cout <= 0 || a->cin % epc || a->ldx % epc) { set_error("vqx_conv: cin %d / ldx %d must be multiples of %d", a->cin, a->ldx, epc); return -1; }
  if (mode == MODE_DGRAD && a->cout % epc) { set_error("vqx_conv_dgrad: cout %d must be a multiple of %d", a->cout, epc); return -1; }
  if (!aligned16(a->x) || !aligned16(a->w)) { set_error("vqx_conv: x/w must be 16-byte aligned"); return -1; }
  if (a->prologue < 0 || a->prologue > 3 || (mode == MODE_DGRAD && a->prologue)) { set_error("vqx_conv: bad prologue %d", a->prologue); return -1; }
  if ((a->epilogue & VQX_EPI_BIAS) && !a->bias) { set_error("vqx_conv: BIAS without bias"); return -1; }
  if ((a->epilogue & VQX_EPI_ROWBIAS) && !a->rowbias) { set_error("vqx_conv: ROWBIAS without rowbias"); return -1; }
  if ((a->epilogue & VQX_EPI_RES) && !a->res) { set_error("vqx_conv: RES without res"); return -1; }
  if ((a->epilogue & VQX_EPI_MASK) && !a->mask) { set_error("vqx_conv: MASK without mask"); return -1; }
  if ((a->epilogue & VQX_EPI_GNADD) && !(a->gn_h && a->gn_mean_rstd && a->gn_gamma && a->gn_beta)) { set_error("vqx_conv: GNADD operands missing"); return -1; }
  if ((a->epilogue & VQX_EPI_SPLIT) && !a->out2) { set_error("vqx_conv: SPLIT without out2"); return -1; }
  if (!a->y) { set_error("vqx_conv: null y"); return -1; }

  GemmParams P = {};
  P.a = a->x; P.b = a->w; P.n_rows = a->n_rows; P.T = a->T; P.lda = a->ldx;
  P.kcin = a->cin; P.K = a->ntaps * a->cin; P.Mc = (int)a->n_rows; P.Nc = a->cout;
  P.ntaps = a->ntaps; P.pad = a->pad; P.sign = 1;
  P.cdim = a->cout;  // DGRAD: cin of the forward layer
  P.pro = a->prologue; P.pro_scale = a->pro_scale;
  P.tiles_m = (int)((a->n_rows + kBM - 1) / kBM); P.tiles_n = (a->cout + kBN - 1) / kBN; P.splits = 1;
  P.y = a->y; P.ldy = a->ldy; P.epi = a->epilogue; P.dtype_out_f32 = (a->epilogue & VQX_EPI_OUTF32) ? 1 : 0;
  P.bias = a->bias; P.rowbias = a->rowbias; P.res = a->res; P.ldres = a->ldres;
  P.mask = a->mask; P.ldmask = a->ldmask; P.mask_slope = a->mask_slope; P.mask_scale = a->mask_scale;
  P.gn_h = a->gn_h; P.ldgn = a->ldgn; P.gn_mr = a->gn_mean_rstd; P.gn_gamma = a->gn_gamma; P.gn_beta = a->gn_beta;
  P.out2 = a->out2; P.ldo2 = a->ldo2; P.split_col = a->split_col; P.out2_acc = a->out2_accumulate;
  const int grid = P.tiles_m * P.tiles_n;
  if (a->dtype == VQX_BF16) {
    if (mode == MODE_FWD) launch_mode<bf16_t, MODE_FWD>(P, grid, s); else launch_mode<bf16_t, MODE_DGRAD>(P, grid, s);
  } else {
    if (mode == MODE_FWD) launch_mode<float, MODE_FWD>(P, grid, s); else launch_mode<float, MODE_DGRAD>(P, grid, s);
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
  if (a->ntaps < 1 || a->ntaps > 3) { set_error("vqx_conv1d_wgrad: ntaps %d", a->ntaps); return -1; }
  if (a->n_rows <= 0 || a->T <= 0 || a->n_rows % a->T) { set_error("vqx_conv1d_wgrad: bad n_rows/T"); return -1; }
  if (a->r_dim % epc || a->c_dim % epc || a->ldp % epc || a->ldq % epc) { set_error("vqx_conv1d_wgrad: dims must be multiples of %d", epc); return -1; }
  if (a->splits < 1) { set_error("vqx_conv1d_wgrad: splits < 1"); return -1; }
  if (!aligned16(a->p) || !aligned16(a->q) || !a->slabs) { set_error("vqx_conv1d_wgrad: bad pointers"); return -1; }
  if (a->shift_sign != 1 && a->shift_sign != -1) { set_error("vqx_conv1d_wgrad: shift_sign must be +-1"); return -1; }
  const int BK = a->dtype == VQX_BF16 ? 64 : 32;
  GemmParams P = {};
  P.a = a->p; P.b = a->q; P.n_rows = a->n_rows; P.T = a->T; P.lda = a->ldp; P.ldb = a->ldq;
  P.Mc = a->r_dim; P.Nc = a->ntaps * a->c_dim; P.ntaps = a->ntaps; P.pad = a->pad; P.sign = a->shift_sign;
  P.cdim = a->c_dim; P.pro = a->q_prologue; P.pro_scale = a->pro_scale;
  P.tiles_m = (P.Mc + kBM - 1) / kBM; P.tiles_n = (P.Nc + kBN - 1) / kBN; P.splits = a->splits;
  int64_t kps = (a->n_rows + a->splits - 1) / a->splits;
  kps = (kps + BK - 1) / BK * BK;
  P.k_per_split = kps;
  P.y = a->slabs;
  const int grid = P.tiles_m * P.tiles_n * P.splits;
  hipStream_t s = (hipStream_t)stream;
  if (a->dtype == VQX_BF16) launch_mode<bf16_t, MODE_WGRAD>(P, grid, s);
  else launch_mode<float, MODE_WGRAD>(P, grid, s);
  return launch_status("vqx_conv1d_wgrad");
}
