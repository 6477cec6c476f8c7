// Ping-pong tap-reuse conv GEMM (3-tap FWD / DGRAD, bf16, T % 256 == 0).
//
// Same tile and LDS images as conv_tr8_kernel: 256*SEGS frames x 128 columns
// per 8-wave workgroup, one workgroup per CU, frames staged once per 32-channel
// stage and read at three row shifts (the taps).  The two 4-wave groups own
// disjoint output rows (SEGS = 2: one 256-frame segment each; SEGS = 1: one
// 128-row half each), so every SIMD hosts one wave of each group.
//
// conv_tr8_kernel runs all eight waves in lockstep: every wave reads its
// fragments, waits, multiplies, and meets the others at the stage barrier, so
// both waves of a SIMD wait on LDS at the same time and the matrix pipe idles
// (its no-DMA variant reaches ~65% of the MFMA rate).  Here the groups
// alternate: the work is cut into units (U per stage; a unit = every tap of
// KS/U 16-channel slices), and in each barrier-delimited segment one group
// multiplies the unit whose fragments it read in the previous segment while
// the other group reads its fragments for the same unit (and issues its
// share of the stage DMAs).  Each SIMD's matrix pipe is then fed by one wave
// while its partner loads.
//
// Segment timeline (group 1 runs one segment behind group 0):
//   seg 0:       G0 load u0                G1 -
//   seg 2i+1:    G0 compute u_i            G1 load u_i
//   seg 2i+2:    G0 load u_{i+1}           G1 compute u_i
// Staging: an NST-deep ring, D = NST-1 stages in flight.  Each wave issues
// its pieces of stage kt+D in its load of unit (kt, 0); the buffer it fills
// held stage kt-1, whose last reader (G1's load of (kt-1, U-1)) finished
// before the barrier that precedes it.  Stage kt+1 must have landed before
// G0 loads (kt+1, 0): every wave waits for it (counted vmcnt) in the segment
// where G0 computes (kt, U-1) and G1 loads it, before that segment's barrier.
// Every load phase ends with lgkmcnt(0), so a segment barrier also retires
// all LDS reads issued before it.
//
// Measured (tools/lab/tr_lab.cpp, profiles/r03/pp_lab_variants.txt): on the
// 512-frame dec_in FWD (512 -> 1024) 45-51 vs 47-55 us for conv_tr8_kernel
// (4-8%), which is where the library uses it (SEGS = 2, U = 2).  SEGS = 1 ran
// level with conv_tr8_kernel / conv_tr_kernel on enc FWD and 5-7% slower on
// the DGRADs; v_mfma_f32_16x16x32_bf16 blocks (one tap per unit) were 2-3%
// slower than the 32x32x16 form (profiles/r03/pp_lab_m16.txt).  With the MFMAs
// removed the load phases alone take ~70% of the full kernel's time, so the
// fragment reads + DMA issue, not the matrix pipe, bound it.
#pragma once
#include "vqx_gemm_kernel.h"

namespace vqx {

// segment barrier: memory operations (asm memory clobber) and MFMAs
// (sched_barrier) stay on their side
__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int SEGS>
__host__ __device__ constexpr int conv_pp_nst() { return SEGS == 2 ? 2 : 3; }

template <int SEGS>
__host__ __device__ constexpr int conv_pp_smem() {
  constexpr int A = ((SEGS * 258 * 64 + 1023) / 1024) * 1024, STAGE = A + 3 * 128 * 64;
  return conv_pp_nst<SEGS>() * STAGE > 2 * 45056 ? conv_pp_nst<SEGS>() * STAGE : 2 * 45056;
}

template <int MODE, int EK, int SEGS, int U>
__global__ __launch_bounds__(512, 1) void conv_pp_kernel(GemmParams P) {
  using T = bf16_t;
  constexpr int BKC = 32, ES = 2, EPC = 8, KCH = BKC * ES / 16;
  constexpr int NST = conv_pp_nst<SEGS>(), D = NST - 1;
  constexpr int SROWS = 258;
  constexpr int AROWS = SEGS * SROWS;
  constexpr int A_PIECES = (AROWS * BKC * ES + 1023) / 1024;
  constexpr int A_BYTES = A_PIECES * 1024;
  constexpr int PWA = (A_PIECES + 7) / 8;
  constexpr int TAP_BYTES = 128 * BKC * ES;
  constexpr int TAP_PIECES = TAP_BYTES / 1024;
  constexpr int B_PIECES = 3 * TAP_PIECES;
  constexpr int PWB = (B_PIECES + 7) / 8;
  constexpr int STAGE = A_BYTES + 3 * TAP_BYTES;
  constexpr int EPI_BYTES = 45056;
  constexpr int KS = BKC / 16;     // 16-channel slices per stage
  constexpr int SPS = KS / U;      // slices per unit
  static_assert(KS % U == 0, "units");
  static_assert(conv_pp_smem<SEGS>() >= NST * STAGE, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[conv_pp_smem<SEGS>()];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2, wm = (wid >> 1) & 1, wn = wid & 1;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lin / P.tiles_n, tn = lin - tm * P.tiles_n;
  const int64_t m0 = (int64_t)tm * (256 * SEGS);
  const int n0 = tn * kBN;
  const int nk = P.kcin / BKC;

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
    aoff[i] = ok ? (unsigned)(((f0 + r) * P.lda + kch * EPC) * ES) : kOOB;
  }
  unsigned boff[PWB];
#pragma unroll
  for (int i = 0; i < PWB; ++i) {
    const int pb = wid + 8 * i;
    const int tap = pb / TAP_PIECES, c = (pb % TAP_PIECES) * 64 + lane;
    if constexpr (MODE == MODE_FWD) {
      const int row = c / KCH, kch = (c % KCH) ^ tr_kswz<KCH>(row);
      const int co = n0 + row;
      boff[i] = (pb < B_PIECES && co < P.Nc) ? (unsigned)(((int64_t)co * P.K + tap * P.kcin + kch * EPC) * ES) : kOOB;
    } else {
      const int krow = c / 16, cch = (c % 16) ^ mn_swz(krow);
      const int ci = n0 + cch * EPC;
      boff[i] = (pb < B_PIECES && ci < P.Nc)
                    ? (unsigned)(((int64_t)krow * 3 * P.cdim + (2 - tap) * P.cdim + ci) * ES) : kOOB;
    }
  }
  const int npw = (A_PIECES - wid + 7) / 8 + (B_PIECES - wid + 7) / 8;  // this wave's DMAs per stage
  const __amdgpu_buffer_rsrc_t rsA = rsrc_at(P.a, -(int64_t)P.lda * ES, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = rsrc_at(P.b, 0, P.b_bytes);

  auto dma_stage = [&](int kt) {
    const int c0 = kt * BKC;
    const unsigned ksa = (unsigned)(c0 * ES);
    const unsigned ksb = MODE == MODE_FWD ? (unsigned)(c0 * ES) : (unsigned)((int64_t)c0 * 3 * P.cdim * ES);
    char* st = smem + (kt % NST) * STAGE;
#pragma unroll
    for (int i = 0; i < PWA; ++i)
      if (wid + 8 * i < A_PIECES) dma16(rsA, st + (wid + 8 * i) * 1024, aoff[i] + ksa);
#pragma unroll
    for (int i = 0; i < PWB; ++i)
      if (wid + 8 * i < B_PIECES) dma16(rsB, st + A_BYTES + (wid + 8 * i) * 1024, boff[i] + ksb);
  };
  // stage kt+1 must have landed; stages kt+2 .. min(kt+D, nk-1) may stay in flight
  auto wait_next = [&](int kt) {
    if constexpr (D == 1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      int ahead = (kt + D < nk - 1 ? kt + D : nk - 1) - (kt + 1);
      wait_vm(ahead > 0 ? ahead * npw : 0);
    }
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
  int qrow[SEGS];
#pragma unroll
  for (int j = 0; j < SEGS; ++j) {
    const int qd = grp * SEGS + j;
    qrow[j] = (qd >> 1) * SROWS + (qd & 1) * 128 + wm * 64 + r32;
  }

  bf16x8_t af[SPS][3][SEGS][2], bfr[SPS][3][2];
  // fragments of unit w of stage kt (LDS -> registers); unit 0 also issues stage kt+D
  auto load = [&](int kt, auto w_c) __attribute__((always_inline)) {
    constexpr int w = decltype(w_c)::value;
    if (w == 0 && kt + D < nk) dma_stage(kt + D);
    const char* la = smem + (kt % NST) * STAGE;
#pragma unroll
    for (int ss = 0; ss < SPS; ++ss) {
      const int s = w * SPS + ss;
#pragma unroll
      for (int tap = 0; tap < 3; ++tap) {
        const char* lb = la + A_BYTES + tap * TAP_BYTES;
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          if constexpr (MODE == MODE_FWD) {
            bfr[ss][tap][x] = *(const bf16x8_t*)(lb + tr_kmaj_off<KCH>(wn * 64 + x * 32 + r32, 2 * s + h));
          } else {
            const int kb = 16 * s + (g >> 1) * 8;
            const int ch = ((wn * 64 + x * 32 + (g & 1) * 16) >> 3) + (p >> 1);
            const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (VQX_LDS(s16x4_t)*)(lb + mnmaj_off<T>(kb + q, ch) + 8 * (p & 1)));
            const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (VQX_LDS(s16x4_t)*)(lb + mnmaj_off<T>(kb + 4 + q, ch) + 8 * (p & 1)));
            const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            bfr[ss][tap][x] = __builtin_bit_cast(bf16x8_t, v);
          }
#pragma unroll
          for (int j = 0; j < SEGS; ++j)
            af[ss][tap][j][x] = *(const bf16x8_t*)(la + tr_kmaj_off<KCH>(qrow[j] + x * 32 + tap, 2 * s + h));
        }
      }
    }
  };
  auto compute = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int ss = 0; ss < SPS; ++ss)
#pragma unroll
      for (int tap = 0; tap < 3; ++tap)
#pragma unroll
        for (int j = 0; j < SEGS; ++j)
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
              acc[j][mi][ni] =
                  __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[ss][tap][ni], af[ss][tap][j][mi], acc[j][mi][ni], 0, 0, 0);
  };

  if (nk > 0) {
    // prologue: stages 0 .. D-1 in flight, stage 0 landed everywhere
#pragma unroll
    for (int t = 0; t < D; ++t)
      if (t < nk) dma_stage(t);
    wait_vm(D > 1 && nk > 1 ? (D - 1 < nk - 1 ? D - 1 : nk - 1) * npw : 0);
    pp_barrier();
    if (grp == 0) {
      load(0, std::integral_constant<int, 0>{});
      pp_barrier();
      for (int kt = 0; kt < nk; ++kt) {
        static_for<U>([&](auto w_c) __attribute__((always_inline)) {
          constexpr int w = decltype(w_c)::value;
          compute();
          if (w == U - 1) wait_next(kt);
          pp_barrier();
          if constexpr (w + 1 < U) load(kt, std::integral_constant<int, w + 1>{});
          else if (kt + 1 < nk) load(kt + 1, std::integral_constant<int, 0>{});
          pp_barrier();
        });
      }
    } else {
      pp_barrier();
      for (int kt = 0; kt < nk; ++kt) {
        static_for<U>([&](auto w_c) __attribute__((always_inline)) {
          constexpr int w = decltype(w_c)::value;
          load(kt, w_c);
          if (w == U - 1) wait_next(kt);
          pp_barrier();
          compute();
          pp_barrier();
        });
      }
    }
  }
#pragma unroll
  for (int j = 0; j < SEGS; ++j)
    tile_epilogue<T, MODE, EK>(P, acc[j], smem + grp * EPI_BYTES, (int)(m0 + (grp * SEGS + j) * 128), n0, tn, 0,
                               P.gn_mr, tid & 255);
}

}  // namespace vqx
