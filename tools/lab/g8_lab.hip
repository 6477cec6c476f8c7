// Lab: a 256 x 256-tile implicit-im2col conv GEMM (FWD, bf16) with 8 waves,
// one workgroup per CU, a 2 x 64 KiB LDS-DMA ring released half-tile by
// half-tile, counted vmcnt waits that keep the next K-tile's loads in flight
// across the barriers, and two barriers per 64-deep K-tile
// (cdna_hip_programming.md "The 256^2 8-phase template": the staging pipeline,
// not the tile alone, is the lever).  Timed against conv_gemm_kernel (128 x 128,
// two workgroups per CU, 2-deep ring drained every K-tile) on the config-2
// shapes; outputs compared bit for bit (same K order per accumulator).
//
// K-tile t lives in buffer t & 1 as four 16-KiB half-tiles: A0 / A1 (frame rows
// 0-127 / 128-255, read by wave group 0 / 1) and B0 / B1 (output channels
// 0-127 / 128-255, read by both groups).  Per K-tile, phases:
//   ph0  issue L(t+1, B1)        read A (all k) + B0 k 0-31   MFMA q0 k 0-31
//   ph1                          read B0 k 32-63              MFMA q0 k 32-63
//        lgkmcnt(0), vmcnt -> L(t, B1) landed, barrier  (A, B0 of t free; B1 of t readable)
//   ph2  issue L(t+2, A0 A1 B0)  read B1 k 0-31               MFMA q1 k 0-31
//   ph3                          read B1 k 32-63              MFMA q1 k 32-63
//        lgkmcnt(0), vmcnt -> L(t+1, A0 A1 B0) landed, barrier (B1 of t free)
// so every half-tile load has ~6 phases (1.5 K-tiles) to land.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "vqx_gemm_inst.h"

using namespace vqx;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

namespace vqx {

constexpr int G8_HALF = 16384;          // one half-tile: 128 rows x 64 bf16
constexpr int G8_BUF = 4 * G8_HALF;     // A0 A1 B0 B1
constexpr int G8_SMEM = 2 * G8_BUF;     // 128 KiB

__device__ __forceinline__ void g8_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ unsigned long long* g8_stamps;  // [block][wave 0 / 4][5]: compute01, wait1, compute23, wait3, total

// LAB: 0 full, 1 no operand DMA (waits kept), 2 no MFMA (fragment reads kept live); PRIO: s_setprio(1) around
// the MFMA clusters; STAMP: s_memtime phase sums of waves 0 and 4
template <int EK, int LAB = 0, bool PRIO = false, bool STAMP = false, bool RA = false>
__global__ __launch_bounds__(512, 1) void g8_fwd_kernel(GemmParams P) {
  using T = bf16_t;
  constexpr int ES = 2, EPC = 8, KCH = 8;
  __shared__ __attribute__((aligned(16))) char smem[G8_SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2, wm = (wid >> 1) & 1, wn = wid & 1;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tn2 = (P.tiles_n + 1) / 2;  // 256-wide column tiles
  const int tm = lin / tn2, tn = lin - tm * tn2;
  const int m0 = tm * 256, n0 = tn * 256;
  const int nk = P.K / 64;  // host: cin % 64 == 0

  // per-thread addressing: pieces 2*wid, 2*wid+1 of each half-tile (16 pieces of 1 KiB)
  unsigned aoff[2][2];  // [A half][piece]
  int amask[2][2];
  unsigned boff[2][2];  // [B half][piece]
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = (2 * wid + i) * 64 + lane;
      const int row = c / KCH, kch = (c % KCH) ^ kswz<KCH>(row);
      const int64_t n = (int64_t)m0 + h * 128 + row;
      const int t = (int)(n % P.T);
      int msk = 0;
      if (n < P.n_rows)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int tt = t + j * P.dil - P.pad;
          msk |= (j < P.ntaps && tt >= 0 && tt < P.T) ? (1 << j) : 0;
        }
      amask[h][i] = msk;
      aoff[h][i] = (unsigned)((n * P.lda + kch * EPC) * ES + (int64_t)P.pad * P.lda * ES);
      const int co = n0 + h * 128 + row;
      boff[h][i] = co < P.Nc ? (unsigned)(((int64_t)co * P.K + kch * EPC) * ES) : kOOB;
    }
  const __amdgpu_buffer_rsrc_t rsA = rsrc_at(P.a, -(int64_t)P.pad * P.lda * ES, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = rsrc_at(P.b, 0, P.b_bytes);

  auto lds_half = [&](int buf, int which) { return smem + buf * G8_BUF + which * G8_HALF + wid * 2048; };
  // which: 0 A0, 1 A1, 2 B0, 3 B1
  auto load_a = [&](int t) {  // both A halves of K-tile t
    if constexpr (LAB == 1) return;
    const int k0 = t * 64;
    const int tap = k0 / P.kcin, c0 = k0 - tap * P.kcin;
    const unsigned ksa = (unsigned)(((tap * P.dil - P.pad) * P.lda + c0) * ES);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        dma16(rsA, lds_half(t & 1, h) + i * 1024, ((amask[h][i] >> tap) & 1) ? aoff[h][i] + ksa : kOOB);
  };
  auto load_b = [&](int t, int h) {
    if constexpr (LAB == 1) return;
    const unsigned ksb = (unsigned)(t * 64 * ES);
#pragma unroll
    for (int i = 0; i < 2; ++i) dma16(rsB, lds_half(t & 1, 2 + h) + i * 1024, boff[h][i] + ksb);
  };

  f32x16_t acc[2][2][2];  // [quadrant (B half)][mi][ni]
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[q][i][j][e] = 0.f;
  const int r32 = lane & 31, h32 = lane >> 5;
  bf16x8_t af[2][4];  // [mi][ks]
  auto read_a = [&](int buf) {
    const char* la = smem + buf * G8_BUF + grp * G8_HALF;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int s = 0; s < 4; ++s) af[x][s] = *(const bf16x8_t*)(la + kmaj_off<KCH>(wm * 64 + x * 32 + r32, 2 * s + h32));
  };
  auto read_b = [&](int buf, int q, int s0, bf16x8_t (&bf)[2][2]) {
    const char* lb = smem + buf * G8_BUF + (2 + q) * G8_HALF;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int s = 0; s < 2; ++s) bf[x][s] = *(const bf16x8_t*)(lb + kmaj_off<KCH>(wn * 64 + x * 32 + r32, 2 * (s0 + s) + h32));
  };
  auto mfma = [&](int q, int s0, const bf16x8_t (&bf)[2][2]) {
    if constexpr (LAB == 2) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int x = 0; x < 2; ++x) asm volatile("" ::"v"(bf[x][s]), "v"(af[x][s0 + s]));
      return;
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[q][mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[ni][s], af[mi][s0 + s], acc[q][mi][ni], 0, 0, 0);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  };
  unsigned long long st[5] = {0, 0, 0, 0, 0}, tm_ = 0;
  auto stamp = [&](int slot) {
    if constexpr (STAMP) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
      if (slot >= 0) st[slot] += now - tm_;
      tm_ = now;
    }
  };
  stamp(-1);
  const unsigned long long t_begin = tm_;

  if (nk > 0) {
    // prologue: K-tile 0 whole, K-tile 1's A and B0; wait for tile 0's A and B0
    load_a(0);
    load_b(0, 0);
    load_b(0, 1);
    if (nk > 1) {
      load_a(1);
      load_b(1, 0);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
    g8_barrier();
    for (int t = 0; t < nk; ++t) {
      const int buf = t & 1;
      bf16x8_t b0[2][2], b1[2][2];
      stamp(-1);
      // ph0
      if (t + 1 < nk) load_b(t + 1, 1);
      if constexpr (RA) {  // every fragment read of ph0 + ph1 issued before the first MFMA
        read_a(buf);
        read_b(buf, 0, 0, b0);
        read_b(buf, 0, 2, b1);
        __builtin_amdgcn_sched_barrier(0);
        mfma(0, 0, b0);
        mfma(0, 2, b1);
      } else {
        read_a(buf);
        read_b(buf, 0, 0, b0);
        mfma(0, 0, b0);
        // ph1
        read_b(buf, 0, 2, b1);
        mfma(0, 2, b1);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      stamp(0);
      // L(t, B1) landed: younger are L(t+1, A, B0) (6) and L(t+1, B1) (2) when t+1 < nk
      if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      g8_barrier();
      stamp(1);
      // ph2
      if (t + 2 < nk) {
        load_a(t + 2);
        load_b(t + 2, 0);
      }
      if constexpr (RA) {
        read_b(buf, 1, 0, b0);
        read_b(buf, 1, 2, b1);
        __builtin_amdgcn_sched_barrier(0);
        mfma(1, 0, b0);
        mfma(1, 2, b1);
      } else {
        read_b(buf, 1, 0, b0);
        mfma(1, 0, b0);
        // ph3
        read_b(buf, 1, 2, b1);
        mfma(1, 2, b1);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      stamp(2);
      // L(t+1, A, B0) landed: younger are L(t+1, B1) (2) and L(t+2, A, B0) (6)
      if (t + 2 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      g8_barrier();
      stamp(3);
    }
  }
  if constexpr (STAMP) {
    stamp(-1);
    st[4] = tm_ - t_begin;
    if (lane == 0 && (wid == 0 || wid == 4)) {
      unsigned long long* o = g8_stamps + ((size_t)blockIdx.x * 2 + (wid >> 2)) * 5;
      for (int i = 0; i < 5; ++i) o[i] = st[i];
    }
  }
  // epilogue: each 4-wave group runs tile_epilogue on its two 128 x 128 quadrants
#pragma unroll
  for (int q = 0; q < 2; ++q)
    tile_epilogue<T, MODE_FWD, EK>(P, acc[q], smem + grp * 45056, m0 + grp * 128, n0 + q * 128, 2 * tn + q, 0,
                                   P.gn_mr, tid & 255);
}

// The same pipeline with v_mfma_f32_16x16x32_bf16 (a 64 x 64 wave tile = 4 x 4 blocks per quadrant):
// MI355X_MICROARCH "DVFS give-back" item 7 -- on random data the chip holds a higher clock on this shape.
// Lab epilogue: direct bf16 stores (4 consecutive channels per lane).
template <bool RA = true>
__global__ __launch_bounds__(512, 1) void g8m16_fwd_kernel(GemmParams P) {
  constexpr int ES = 2, EPC = 8, KCH = 8;
  __shared__ __attribute__((aligned(16))) char smem[G8_SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2, wm = (wid >> 1) & 1, wn = wid & 1;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tn2 = (P.tiles_n + 1) / 2;
  const int tm = lin / tn2, tn = lin - tm * tn2;
  const int m0 = tm * 256, n0 = tn * 256;
  const int nk = P.K / 64;
  unsigned aoff[2][2];
  int amask[2][2];
  unsigned boff[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = (2 * wid + i) * 64 + lane;
      const int row = c / KCH, kch = (c % KCH) ^ kswz<KCH>(row);
      const int64_t n = (int64_t)m0 + h * 128 + row;
      const int t = (int)(n % P.T);
      int msk = 0;
      if (n < P.n_rows)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int tt = t + j * P.dil - P.pad;
          msk |= (j < P.ntaps && tt >= 0 && tt < P.T) ? (1 << j) : 0;
        }
      amask[h][i] = msk;
      aoff[h][i] = (unsigned)((n * P.lda + kch * EPC) * ES + (int64_t)P.pad * P.lda * ES);
      const int co = n0 + h * 128 + row;
      boff[h][i] = co < P.Nc ? (unsigned)(((int64_t)co * P.K + kch * EPC) * ES) : kOOB;
    }
  const __amdgpu_buffer_rsrc_t rsA = rsrc_at(P.a, -(int64_t)P.pad * P.lda * ES, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = rsrc_at(P.b, 0, P.b_bytes);
  auto lds_half = [&](int buf, int which) { return smem + buf * G8_BUF + which * G8_HALF + wid * 2048; };
  auto load_a = [&](int t) {
    const int k0 = t * 64;
    const int tap = k0 / P.kcin, c0 = k0 - tap * P.kcin;
    const unsigned ksa = (unsigned)(((tap * P.dil - P.pad) * P.lda + c0) * ES);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        dma16(rsA, lds_half(t & 1, h) + i * 1024, ((amask[h][i] >> tap) & 1) ? aoff[h][i] + ksa : kOOB);
  };
  auto load_b = [&](int t, int h) {
    const unsigned ksb = (unsigned)(t * 64 * ES);
#pragma unroll
    for (int i = 0; i < 2; ++i) dma16(rsB, lds_half(t & 1, 2 + h) + i * 1024, boff[h][i] + ksb);
  };
  f32x4_t acc[2][4][4];  // [quadrant][mi][ni]
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[q][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int r16 = lane & 15, g4 = lane >> 4;
  bf16x8_t af[4][2];  // [mi][ks]
  auto read_a = [&](int buf) {
    const char* la = smem + buf * G8_BUF + grp * G8_HALF;
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int s = 0; s < 2; ++s) af[x][s] = *(const bf16x8_t*)(la + kmaj_off<KCH>(wm * 64 + x * 16 + r16, 4 * s + g4));
  };
  auto read_b = [&](int buf, int q, int s, bf16x8_t (&bf)[4]) {
    const char* lb = smem + buf * G8_BUF + (2 + q) * G8_HALF;
#pragma unroll
    for (int x = 0; x < 4; ++x) bf[x] = *(const bf16x8_t*)(lb + kmaj_off<KCH>(wn * 64 + x * 16 + r16, 4 * s + g4));
  };
  auto mfma = [&](int q, int s, const bf16x8_t (&bf)[4]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        acc[q][mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ni], af[mi][s], acc[q][mi][ni], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  if (nk > 0) {
    load_a(0);
    load_b(0, 0);
    load_b(0, 1);
    if (nk > 1) {
      load_a(1);
      load_b(1, 0);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
    g8_barrier();
    for (int t = 0; t < nk; ++t) {
      const int buf = t & 1;
      bf16x8_t b0[4], b1[4];
      if (t + 1 < nk) load_b(t + 1, 1);
      read_a(buf);
      read_b(buf, 0, 0, b0);
      read_b(buf, 0, 1, b1);
      if constexpr (RA) __builtin_amdgcn_sched_barrier(0);
      mfma(0, 0, b0);
      mfma(0, 1, b1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      g8_barrier();
      if (t + 2 < nk) {
        load_a(t + 2);
        load_b(t + 2, 0);
      }
      read_b(buf, 1, 0, b0);
      read_b(buf, 1, 1, b1);
      if constexpr (RA) __builtin_amdgcn_sched_barrier(0);
      mfma(1, 0, b0);
      mfma(1, 1, b1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (t + 2 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      g8_barrier();
    }
  }
  // lab epilogue: D[channel 4*g4 + r][frame r16] of block (mi, ni) -> y[frame][channel]
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int64_t row = (int64_t)m0 + grp * 128 + wm * 64 + mi * 16 + r16;
        const int col = n0 + q * 128 + wn * 64 + ni * 16 + 4 * g4;
        if (row < P.n_rows && col < P.Nc) {
          uint2 pk;
          pk.x = pack_bf16x2(acc[q][mi][ni][0], acc[q][mi][ni][1]);
          pk.y = pack_bf16x2(acc[q][mi][ni][2], acc[q][mi][ni][3]);
          *(uint2*)((bf16_t*)P.y + row * P.ldy + col) = pk;
        }
      }
}

}  // namespace vqx

static float time_us(const void* fn, int grid, int block, GemmParams P, int reps) {
  void* args[] = {(void*)&P};
  for (int i = 0; i < 3; ++i) CK(hipLaunchKernel(fn, dim3(grid), dim3(block), args, 0, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) CK(hipLaunchKernel(fn, dim3(grid), dim3(block), args, 0, 0));
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 1e3f * ms / reps;
}

int main() {
  const int64_t N = 16384;
  const int T = 256;
  struct Case {
    const char* name;
    int cin, cout, ntaps;
  } cases[] = {
      {"dec_in_fwd 512->1024 k3", 512, 1024, 3},
      {"enc_k3_fwd 512->512 k3", 512, 512, 3},
      {"enc_sk_fwd 512->512 k1", 512, 512, 1},
      {"dec_rs_fwd 512->640 k1", 512, 640, 1},
      {"k1 1536->1024", 1536, 1024, 1},
  };
  std::vector<unsigned short> h((size_t)N * 1536);
  unsigned r = 12345u;
  for (auto& v : h) {  // bf16 uniform-ish in +-[0.5, 1) with random signs: random data (MFMA clocks)
    r = r * 1664525u + 1013904223u;
    v = (unsigned short)(0x3f00 + ((r >> 9) & 0x7f)) | ((r >> 20) & 1 ? 0x8000 : 0);
  }
  void *x, *w, *y0, *y1;
  CK(hipMalloc(&x, (size_t)N * 1536 * 2));
  CK(hipMalloc(&w, (size_t)1024 * 1536 * 3 * 2));
  CK(hipMalloc(&y0, (size_t)N * 1024 * 2));
  CK(hipMalloc(&y1, (size_t)N * 1024 * 2));
  CK(hipMemcpy(x, h.data(), (size_t)N * 1536 * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, h.data(), (size_t)1024 * 1536 * 2, hipMemcpyHostToDevice));
  int dev = 0, cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  for (const Case& c : cases) {
    GemmParams P = {};
    P.a = x;
    P.b = w;
    P.a_bytes = (int64_t)N * c.cin * 2;
    P.b_bytes = (int64_t)c.cout * c.ntaps * c.cin * 2;
    P.n_rows = N;
    P.T = T;
    P.lda = c.cin;
    P.kcin = c.cin;
    P.K = c.ntaps * c.cin;
    P.Mc = (int)N;
    P.Nc = c.cout;
    P.ntaps = c.ntaps;
    P.pad = (c.ntaps - 1) / 2;
    P.sign = 1;
    P.dil = 1;
    P.cdim = c.cout;
    P.tiles_n = (c.cout + 127) / 128;
    P.tiles_m = (int)(N / 128);
    P.splits = 1;
    P.ldy = c.cout;
    P.epi = 0;
    const double fl = 2.0 * N * P.K * c.cout;
    // reference: conv_gemm_kernel (implicit im2col, 128 x 128, 2 per CU)
    P.y = y0;
    const void* ref = (const void*)conv_gemm_kernel<bf16_t, MODE_FWD, VQX_PRO_NONE, false, 64, 2, EK_NONE>;
    const float t_ref = time_us(ref, P.tiles_m * P.tiles_n, 256, P, 20);
    P.y = y1;
    const int grid8 = (int)(N / 256) * ((c.cout + 255) / 256);
    const float t_g8 = time_us((const void*)g8_fwd_kernel<EK_NONE>, grid8, 512, P, 20);
    const float t_nodma = time_us((const void*)g8_fwd_kernel<EK_NONE, 1>, grid8, 512, P, 20);
    const float t_nomfma = time_us((const void*)g8_fwd_kernel<EK_NONE, 2>, grid8, 512, P, 20);
    const float t_prio = time_us((const void*)g8_fwd_kernel<EK_NONE, 0, true>, grid8, 512, P, 20);
    const float t_ra = time_us((const void*)g8_fwd_kernel<EK_NONE, 0, true, false, true>, grid8, 512, P, 20);
    const float t_ra0 = time_us((const void*)g8_fwd_kernel<EK_NONE, 1, true, false, true>, grid8, 512, P, 20);
    unsigned long long* stb;
    CK(hipMalloc(&stb, (size_t)grid8 * 2 * 5 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g8_stamps), &stb, sizeof(stb)));
    const float t_st = time_us((const void*)g8_fwd_kernel<EK_NONE, 0, false, true>, grid8, 512, P, 3);
    std::vector<unsigned long long> hs((size_t)grid8 * 2 * 5);
    CK(hipMemcpy(hs.data(), stb, hs.size() * 8, hipMemcpyDeviceToHost));
    CK(hipFree(stb));
    double sum[5] = {0, 0, 0, 0, 0};
    for (int b = 0; b < grid8 * 2; ++b)
      for (int i = 0; i < 5; ++i) sum[i] += (double)hs[(size_t)b * 5 + i];
    const double tot = sum[4] > 0 ? sum[4] : 1;
    printf("   g8 setprio+read-ahead %.1f us (no DMA %.1f us)\n", t_ra, t_ra0);
    {
      P.y = y1;
      CK(hipMemset(y1, 0, (size_t)N * c.cout * 2));
      const float t16 = time_us((const void*)g8m16_fwd_kernel<true>, grid8, 512, P, 20);
      const float t16n = time_us((const void*)g8m16_fwd_kernel<false>, grid8, 512, P, 20);
      const size_t n = (size_t)N * c.cout;
      std::vector<unsigned short> a(n), b(n);
      CK(hipMemcpy(a.data(), y0, n * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), y1, n * 2, hipMemcpyDeviceToHost));
      size_t d1 = 0, dbig = 0;
      for (size_t i = 0; i < n; ++i) {
        const int d = abs((int)(a[i] & 0x7fff) - (int)(b[i] & 0x7fff)) + ((a[i] ^ b[i]) & 0x8000 ? 1 : 0);
        d1 += a[i] != b[i];
        dbig += d > 1;
      }
      printf("   g8 16x16x32 %.1f us %.1f TF (no read-ahead %.1f us); differing %zu, by > 1 bf16 ulp %zu of %zu\n", t16,
             fl / t16 / 1e6, t16n, d1, dbig, n);
    }
    printf("   g8 ablations: no-DMA %.1f us, no-MFMA %.1f us, setprio %.1f us; stamped %.1f us: "
           "compute01 %.2f wait1 %.2f compute23 %.2f wait3 %.2f of the wave's time (memtime %.0f per wave)\n",
           t_nodma, t_nomfma, t_prio, t_st, sum[0] / tot, sum[1] / tot, sum[2] / tot, sum[3] / tot, tot / (grid8 * 2));
    const size_t n = (size_t)N * c.cout;
    std::vector<unsigned short> a(n), b(n);
    CK(hipMemcpy(a.data(), y0, n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), y1, n * 2, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) bad += a[i] != b[i];
    printf("%-26s conv_gemm %7.1f us %7.1f TF | g8 (grid %d, %d CUs) %7.1f us %7.1f TF | mismatches %zu\n", c.name,
           t_ref, fl / t_ref / 1e6, grid8, cus, t_g8, fl / t_g8 / 1e6, bad);
  }
  return 0;
}
