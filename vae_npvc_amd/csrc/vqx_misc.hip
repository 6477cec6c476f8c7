// Weight norm, GroupNorm (+gated unit), layout, loss, embedding and optimizer
// kernels of the VQ-VAE training step (gfx950).  All reductions are
// deterministic fixed-shape trees (no float atomics), so a step is bitwise
// reproducible apart from the EMA scatter statistics of vq_forward.
#include "vqx_common.h"
#include "vqx_gn_math.h"
#include <math.h>

#include <algorithm>

namespace vqx {

constexpr float kLog2Pi = 1.8378770664093453f;  // log(2*pi), layers.py:8

// ------------------------------------------------------------- weight norm
// torch.nn.utils.weight_norm(dim=0): w = v * (g / ||v||), norm over all dims
// but 0.  Conv1d: v[cout][cin][k], row o = co.  ConvT: v[cin][cout][k], row
// o = ci, effective tap j' = k-1-j.  Packed effective weight:
// wp[co][j*cin + ci].
// Row norms of the ConvTranspose layers (rows = cin, contiguous cout*k):
// one 256-thread block per row, thread t the elements 4t + 1024u + (0..3)
// summed in u order as fmaf(x0, x0, fmaf(x1, x1, fmaf(x2, x2, fmaf(x3, x3, s)))),
// then the block sum: the order adam_wn_kernel uses, so both give the same
// bits.  Conv1d layers get theirs in the pack.
__global__ __launch_bounds__(256) void wn_norm_kernel(const vqx_wn_layer* __restrict__ L, int n_layers) {
  const vqx_wn_layer& l = L[blockIdx.y];
  if (l.kind != 1 || !l.g) return;
  const int o = blockIdx.x;
  if (o >= l.cin) return;
  __shared__ float red[16];
  const int cols = l.cout * l.k;
  const float* v = l.v + (int64_t)o * cols;
  float s = 0.f;
  if ((cols & 3) == 0 && (((uintptr_t)v) & 15) == 0 && cols <= 4096) {
    // the thread's 16-B loads all in flight before the first add
    f32x4_t xv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      xv[u] = 1024 * u < cols ? *(const f32x4_t*)(v + min((int)threadIdx.x * 4 + 1024 * u, cols - 4))
                              : f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x4_t x = xv[u];
      if ((int)threadIdx.x * 4 + 1024 * u < cols)
        s = fmaf(x[0], x[0], fmaf(x[1], x[1], fmaf(x[2], x[2], fmaf(x[3], x[3], s))));
    }
  } else {
    for (int i = threadIdx.x; i < cols; i += 256) s = fmaf(v[i], v[i], s);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) l.norm[o] = sqrtf(s);
}

// Pack w = g*v/||v|| into the effective-conv layout wp[co][j][ci].
// kind 0 (Conv1d, v[co][ci][j]), K > 1: block = one row co: the row is read
//   contiguously into LDS, its norm reduced there (and saved), then written
//   transposed [j][ci] with coalesced stores.
// kind 0, K = 1: no transpose: block = 4 rows, one wave each (16-B loads, a
//   wave reduction, then the scaled row re-read from cache and stored 8 B a
//   lane) -- no LDS, no barriers.
// kind 1 (ConvT, v[ci][co][K-1-j]): block = a 64 ci x TCO co tile, read row
//   segments (TCO*K contiguous floats per ci; 384 B for K = 3) into LDS, write
//   wp[co][j][ci0..] rows of 64 consecutive ci, 16 B a lane.
// The grid is flat over every layer's units (WnUnits: per-layer prefix), so
// no workgroup of a small layer launches only to exit.
constexpr int kWnRow = 4096;
constexpr int kWnMaxL = 256;  // layers per launch (the host launches larger tables in chunks; 1 KiB of kernel argument)
struct WnUnits {
  int n;
  int off[kWnMaxL + 1];
};
// ConvT pack tile width in co: the LDS tile holds 64 ci x (TCO*K + pad) floats
__host__ __device__ inline int wn_tco(int K) { return K <= 3 ? 32 : K <= 4 ? 16 : (K <= 64 ? 64 / K : 1); }
constexpr int kWnBuf = 96 * 65;  // floats: the K = 3 ConvT tile (>= kWnRow + 64 for the Conv1d rows)
static_assert(kWnBuf >= kWnRow + 64, "wn pack LDS");
__host__ __device__ inline int wn_pack_units(const vqx_wn_layer& l) {
  if (l.kind == VQX_WN_RESAMPLE) return l.cout;
  if (l.kind == VQX_WN_RESAMPLE_T) return l.cin;
  if (l.kind == 0) return l.k == 1 ? (l.cout + 3) / 4 : l.cout;
  return ((l.cin + 63) / 64) * ((l.cout + wn_tco(l.k) - 1) / wn_tco(l.k));
}
// one unit of the flat grid (bid: the block's index in it); buf = kWnBuf
// floats of LDS (16-B aligned), red = 16
__device__ __forceinline__ void wn_pack_block(const vqx_wn_layer* __restrict__ L, const WnUnits& U, int bid,
                                              float* __restrict__ buf, float* __restrict__ red) {
  int lo = 0, hi = U.n - 1;  // the layer owning this block: largest li with off[li] <= bid
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (U.off[mid] <= bid) lo = mid; else hi = mid - 1;
  }
  const vqx_wn_layer& l = L[lo];
  const int unit = bid - U.off[lo];
  const int K = l.k, cin = l.cin, cout = l.cout;
  if (l.kind == VQX_WN_RESAMPLE || l.kind == VQX_WN_RESAMPLE_T) {
    // strided conv (include/vqx.h): row r of v, norm, then the folded 3-tap row
    // w_packed[r][m][q*C + c] = w[r][c][S*(m-1) + q + pad]
    const int rows = l.kind == VQX_WN_RESAMPLE ? cout : cin, C = l.kind == VQX_WN_RESAMPLE ? cin : cout;
    const int r = unit;
    if (r >= rows) return;
    const int cols = C * K;
    const float* v = l.v + (int64_t)r * cols;
    float s = 0.f;
    for (int i = threadIdx.x; i < cols; i += 256) {
      const float x = v[i];
      buf[i] = x;
      s = fmaf(x, x, s);
    }
    s = block_sum(s, red);
    float sc = 1.f;
    if (l.g) {
      const float nrm = sqrtf(s);
      if (threadIdx.x == 0) l.norm[r] = nrm;
      sc = l.g[r] / nrm;
    }
    const int S = l.stride, SC = S * C, W = 3 * SC;
    for (int e = threadIdx.x; e < W; e += 256) {
      const int m = e / SC, rem = e - m * SC, q = rem / C, c = rem - q * C;
      const int j = S * (m - 1) + q + l.pad;
      st_dt(l.w_packed, (int64_t)r * W + e, (j >= 0 && j < K) ? buf[c * K + j] * sc : 0.f, l.dtype);
    }
    return;
  }
  if (l.kind == 0 && K == 1) {
    const int co = unit * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (co >= cout) return;
    const float* v = l.v + (int64_t)co * cin;
    const bool vec = (cin & 3) == 0 && (((uintptr_t)v) & 15) == 0 &&
                     ((((uintptr_t)l.w_packed) + (int64_t)co * cin * (l.dtype == VQX_BF16 ? 2 : 4)) & 15) == 0;
    float s = 0.f;
    if (vec) {
      for (int i = lane * 4; i < cin; i += 256) {
        const f32x4_t x = *(const f32x4_t*)(v + i);
        s = fmaf(x[0], x[0], fmaf(x[1], x[1], fmaf(x[2], x[2], fmaf(x[3], x[3], s))));
      }
    } else {
      for (int i = lane; i < cin; i += 64) s = fmaf(v[i], v[i], s);
    }
    s = wave_sum(s);
    float sc = 1.f;
    if (l.g) {
      const float nrm = sqrtf(s);
      if (lane == 0) l.norm[co] = nrm;
      sc = l.g[co] / nrm;
    }
    if (vec) {
      for (int i = lane * 4; i < cin; i += 256) {
        const f32x4_t x = *(const f32x4_t*)(v + i);
        if (l.dtype == VQX_BF16) {
          *(uint2*)((bf16_t*)l.w_packed + (int64_t)co * cin + i) =
              make_uint2(pack_bf16x2(x[0] * sc, x[1] * sc), pack_bf16x2(x[2] * sc, x[3] * sc));
        } else {
          *(f32x4_t*)((float*)l.w_packed + (int64_t)co * cin + i) = f32x4_t{x[0] * sc, x[1] * sc, x[2] * sc, x[3] * sc};
        }
      }
    } else {
      for (int i = lane; i < cin; i += 64) st_dt(l.w_packed, (int64_t)co * cin + i, v[i] * sc, l.dtype);
    }
    return;
  }
  if (l.kind == 0) {
    const int co = unit;
    if (co >= cout) return;
    const int cols = cin * K;
    const float* v = l.v + (int64_t)co * cols;
    float s = 0.f;
    // the row's loads all in flight before the first use (a load + use per
    // iteration of a runtime-bound loop paid one memory latency each)
    if ((cols & 3) == 0 && (((uintptr_t)v) & 15) == 0) {
      // 16-B partition: thread t holds elements 4t + 1024u + (0..3), summed in
      // u order as fmaf(x0, x0, fmaf(x1, x1, fmaf(x2, x2, fmaf(x3, x3, s)))):
      // the order adam_wn_kernel uses for the row norms it writes, so both give
      // the same bits
      f32x4_t xv[kWnRow / 1024];
#pragma unroll
      for (int u = 0; u < kWnRow / 1024; ++u)
        xv[u] = 1024 * u < cols ? *(const f32x4_t*)(v + min((int)threadIdx.x * 4 + 1024 * u, cols - 4))
                                : f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < kWnRow / 1024; ++u) {
        const int i = (int)threadIdx.x * 4 + 1024 * u;
        if (i < cols) {
          const f32x4_t x = xv[u];
          *(f32x4_t*)(buf + i) = x;
          s = fmaf(x[0], x[0], fmaf(x[1], x[1], fmaf(x[2], x[2], fmaf(x[3], x[3], s))));
        }
      }
    } else {
      float xr[kWnRow / 256];
#pragma unroll
      for (int u = 0; u < kWnRow / 256; ++u)
        xr[u] = 256 * u < cols ? v[min((int)threadIdx.x + 256 * u, cols - 1)] : 0.f;
#pragma unroll
      for (int u = 0; u < kWnRow / 256; ++u) {
        const int i = threadIdx.x + 256 * u;
        if (i < cols) {
          buf[i] = xr[u];
          s = fmaf(xr[u], xr[u], s);
        }
      }
    }
    s = block_sum(s, red);  // includes the barriers that publish buf
    float sc = 1.f;
    if (l.g) {
      const float nrm = sqrtf(s);
      if (threadIdx.x == 0) l.norm[co] = nrm;
      sc = l.g[co] / nrm;
    }
    bf16_t* wb = (bf16_t*)l.w_packed + (int64_t)co * cols;
    if (l.dtype == VQX_BF16 && (cin & 3) == 0 && (((uintptr_t)wb) & 7) == 0) {
      for (int e = threadIdx.x * 4; e < cols; e += 1024) {  // 4 consecutive ci of one tap, 8 B a lane
        const int j = e / cin, ci = e - j * cin;
        const float* b = buf + ci * K + j;
        *(uint2*)(wb + e) = make_uint2(pack_bf16x2(b[0] * sc, b[K] * sc), pack_bf16x2(b[2 * K] * sc, b[3 * K] * sc));
      }
      return;
    }
    for (int e = threadIdx.x; e < cols; e += 256) {  // e = j*cin + ci
      const int j = e / cin, ci = e - j * cin;
      st_dt(l.w_packed, (int64_t)co * cols + e, buf[ci * K + j] * sc, l.dtype);
    }
    return;
  }
  // kind 1: tile of 64 ci x TCO co (x K taps) = 64 x TCO*K floats in LDS ([co_local*K + tap][ci], +1 pad)
  const int TCO = wn_tco(K);
  const int ntc = (cout + TCO - 1) / TCO;
  const int ci0 = (unit / ntc) * 64, co0 = (unit % ntc) * TCO;
  if (ci0 >= cin || K > 64) return;
  const int wseg = TCO * K;  // floats per ci row segment (contiguous in v)
  const bool full = ci0 + 64 <= cin && co0 + TCO <= cout;
  constexpr int kTileV4 = 6;  // 16-B loads per thread of a full tile: 64 x wseg floats, wseg <= 96
  if (full && (wseg & 3) == 0 && ((cout * K) & 3) == 0 && (((uintptr_t)l.v) & 15) == 0 && 64 * wseg <= kTileV4 * 1024) {
    const int w4 = wseg >> 2;
    // all of the thread's loads (row segments, gains, norms) in flight at once
    f32x4_t xv[kTileV4];
    float gs[kTileV4], ns[kTileV4];
    const float* __restrict__ gp = l.g;
    const float* __restrict__ np = l.norm;
#pragma unroll
    for (int u = 0; u < kTileV4; ++u) {
      const int e = min((int)threadIdx.x + 256 * u, 64 * w4 - 1), r = e / w4, q = (e - r * w4) * 4;
      const int ci = ci0 + r;
      xv[u] = 256 * u < 64 * w4 ? *(const f32x4_t*)(l.v + ((int64_t)ci * cout + co0) * K + q) : f32x4_t{0.f, 0.f, 0.f, 0.f};
      gs[u] = gp && 256 * u < 64 * w4 ? gp[ci] : 1.f;
      ns[u] = gp && 256 * u < 64 * w4 ? np[ci] : 1.f;
    }
#pragma unroll
    for (int u = 0; u < kTileV4; ++u) {
      const int e = threadIdx.x + 256 * u;
      if (e < 64 * w4) {
        const int r = e / w4, q = (e - r * w4) * 4;
        f32x4_t x = xv[u];
        if (gp) {
          const float sc = gs[u] / ns[u];
          x = f32x4_t{x[0] * sc, x[1] * sc, x[2] * sc, x[3] * sc};
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) buf[(q + k) * 65 + r] = x[k];
      }
    }
  } else {
    for (int e = threadIdx.x; e < 64 * wseg; e += 256) {
      const int r = e / wseg, q = e - r * wseg;  // r: ci offset, q = co_local*K + tap
      const int ci = ci0 + r, co = co0 + q / K;
      float x = 0.f;
      if (ci < cin && co < cout) {
        x = l.v[((int64_t)ci * cout + co0) * K + q];
        if (l.g) x *= l.g[ci] / l.norm[ci];
      }
      buf[q * 65 + r] = x;
    }
  }
  __syncthreads();
  const size_t es = l.dtype == VQX_BF16 ? 2 : 4;
  if (full && (cin & 7) == 0 && (((uintptr_t)l.w_packed) & 15) == 0) {
    for (int e = threadIdx.x; e < wseg * 8; e += 256) {  // e = (co_local*K + j)*8 + 8-ci chunk
      const int cj = e >> 3, r8 = (e & 7) * 8;
      const int cl = cj / K, j = cj - cl * K;
      const float* src = buf + (cl * K + (K - 1 - j)) * 65 + r8;
      const int64_t o = ((int64_t)(co0 + cl) * K + j) * cin + ci0 + r8;
      if (es == 2) {
        *(uint4*)((bf16_t*)l.w_packed + o) = make_uint4(pack_bf16x2(src[0], src[1]), pack_bf16x2(src[2], src[3]),
                                                        pack_bf16x2(src[4], src[5]), pack_bf16x2(src[6], src[7]));
      } else {
        *(f32x4_t*)((float*)l.w_packed + o) = f32x4_t{src[0], src[1], src[2], src[3]};
        *(f32x4_t*)((float*)l.w_packed + o + 4) = f32x4_t{src[4], src[5], src[6], src[7]};
      }
    }
  } else {
    for (int e = threadIdx.x; e < TCO * K * 64; e += 256) {  // e = (co_local*K + j)*64 + ci_local
      const int cj = e >> 6, r = e & 63;
      const int cl = cj / K, j = cj - cl * K;
      const int co = co0 + cl, ci = ci0 + r;
      if (co < cout && ci < cin)
        st_dt(l.w_packed, ((int64_t)co * K + j) * cin + ci, buf[(cl * K + (K - 1 - j)) * 65 + r], l.dtype);
    }
  }
}
__global__ __launch_bounds__(256) void wn_pack_kernel(const vqx_wn_layer* __restrict__ L, WnUnits U) {
  __shared__ __attribute__((aligned(16))) float buf[kWnBuf];
  __shared__ float red[16];
  wn_pack_block(L, U, (int)blockIdx.x, buf, red);
}

// Sum over splits sp0, sp0+step, ... < splits of the 4 slab values at element
// offset p (slab stride `ss`): NF loads issued before any add, added in split
// order into one accumulator (fixed order: deterministic).
#ifndef VQX_WN_NF  // loads in flight per thread
#define VQX_WN_NF 4
#endif
#ifndef VQX_WN_THREADS  // threads per row block: the slab stream is bound by the loads in flight per CU
#define VQX_WN_THREADS 256
#endif
constexpr int kWnNF = VQX_WN_NF;
constexpr int kWnThreads = VQX_WN_THREADS;
static_assert(kWnThreads == 256, "vqx_gemm_kernel.h wgrad_tile_fixup reproduces the split grouping of 256-thread blocks");
template <bool BF>
__device__ __forceinline__ f32x4_t slab_sum(const void* slabs, int64_t p, int64_t ss, int sp0, int step, int splits) {
  typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
  auto cvt = [](u32x2_t u) -> f32x4_t {
    return {__uint_as_float(u[0] << 16), __uint_as_float(u[0] & 0xffff0000u), __uint_as_float(u[1] << 16),
            __uint_as_float(u[1] & 0xffff0000u)};
  };
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  int sp = sp0;
  if constexpr (BF) {
    const unsigned short* sl = (const unsigned short*)slabs;
    for (; sp + (kWnNF - 1) * step < splits; sp += kWnNF * step) {
      u32x2_t t[kWnNF];
#pragma unroll
      for (int u = 0; u < kWnNF; ++u) t[u] = *(const u32x2_t*)(sl + p + (int64_t)(sp + u * step) * ss);
#pragma unroll
      for (int u = 0; u < kWnNF; ++u) acc += cvt(t[u]);
    }
    u32x2_t t[kWnNF];
#pragma unroll
    for (int u = 0; u < kWnNF - 1; ++u)
      if (sp + u * step < splits) t[u] = *(const u32x2_t*)(sl + p + (int64_t)(sp + u * step) * ss);
#pragma unroll
    for (int u = 0; u < kWnNF - 1; ++u)
      if (sp + u * step < splits) acc += cvt(t[u]);
  } else {
    const float* sl = (const float*)slabs;
    for (; sp + (kWnNF - 1) * step < splits; sp += kWnNF * step) {
      f32x4_t t[kWnNF];
#pragma unroll
      for (int u = 0; u < kWnNF; ++u) t[u] = *(const f32x4_t*)(sl + p + (int64_t)(sp + u * step) * ss);
#pragma unroll
      for (int u = 0; u < kWnNF; ++u) acc += t[u];
    }
    f32x4_t t[kWnNF];
#pragma unroll
    for (int u = 0; u < kWnNF - 1; ++u)
      if (sp + u * step < splits) t[u] = *(const f32x4_t*)(sl + p + (int64_t)(sp + u * step) * ss);
#pragma unroll
    for (int u = 0; u < kWnNF - 1; ++u)
      if (sp + u * step < splits) acc += t[u];
  }
  return acc;
}
// slab_sum<true> (splits 0, 1, ... in order) of two column groups at once,
// p0 and p1: twice the loads in flight.  Buffer loads through one descriptor
// over the slabs (slab bytes < 2^31, caller-checked): a VGPR offset per
// column and the split's offset in an SGPR, where flat loads would hold a
// 64-bit address per load (84 VGPRs: five waves per SIMD instead of eight).
__device__ __forceinline__ void slab_sum2_bf(const void* slabs, int sbytes, int64_t p0, int64_t p1, int64_t ss,
                                             int splits, f32x4_t& a0, f32x4_t& a1) {
  typedef int i32x2_t __attribute__((ext_vector_type(2)));
  auto cvt = [](i32x2_t u) -> f32x4_t {
    return {__uint_as_float((unsigned)u[0] << 16), __uint_as_float((unsigned)u[0] & 0xffff0000u),
            __uint_as_float((unsigned)u[1] << 16), __uint_as_float((unsigned)u[1] & 0xffff0000u)};
  };
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)slabs, (short)0, sbytes, 0x00020000);
  const int v0 = (int)(p0 * 2), v1 = (int)(p1 * 2), sstep = (int)(ss * 2);
  a0 = f32x4_t{0.f, 0.f, 0.f, 0.f};
  a1 = a0;
  int sp = 0;
  for (; sp + kWnNF - 1 < splits; sp += kWnNF) {
    i32x2_t t0[kWnNF], t1[kWnNF];
#pragma unroll
    for (int u = 0; u < kWnNF; ++u) {
      t0[u] = __builtin_amdgcn_raw_buffer_load_b64(rs, v0, (sp + u) * sstep, 0);
      t1[u] = __builtin_amdgcn_raw_buffer_load_b64(rs, v1, (sp + u) * sstep, 0);
    }
#pragma unroll
    for (int u = 0; u < kWnNF; ++u) {
      a0 += cvt(t0[u]);
      a1 += cvt(t1[u]);
    }
  }
  i32x2_t t0[kWnNF], t1[kWnNF];
#pragma unroll
  for (int u = 0; u < kWnNF - 1; ++u)
    if (sp + u < splits) {
      t0[u] = __builtin_amdgcn_raw_buffer_load_b64(rs, v0, (sp + u) * sstep, 0);
      t1[u] = __builtin_amdgcn_raw_buffer_load_b64(rs, v1, (sp + u) * sstep, 0);
    }
#pragma unroll
  for (int u = 0; u < kWnNF - 1; ++u)
    if (sp + u < splits) {
      a0 += cvt(t0[u]);
      a1 += cvt(t1[u]);
    }
}

// Backward per weight-norm row o.  slabs[s][o][x] with x = j*cin+ci (Conv1d,
// row co) or x = j'*cout+co (ConvT, row ci); dW of the effective conv.
// The split-K slabs (fp32, or bf16 in bf16 runs) are summed in fp32 with
// 16-B (8-B) loads, several splits in flight per thread, scattered into the
// row's (c, j) order in LDS, then the norm gradient is formed from LDS and the
// row of v held in registers.  One kWnThreads-thread block per row over a flat
// grid of every layer's rows (WnUnits): the big layers have only 512-640 rows,
// so the block -- not the grid -- must carry the loads in flight.
constexpr int kWnVRegs = 4096 / kWnThreads;  // v row values per thread (row length <= 4096)
constexpr int kWnCrCols = 32;  // columns per column-reduce block
// 16-B column groups per lane on the wave-per-row path (rows <= 256 columns:
// the conditioning linears' 128).  Four (rows <= 1024) cost the whole kernel
// 86 VGPRs, i.e. five waves per SIMD and 5/8 of the slab loads in flight; one
// keeps it at 64 VGPRs, eight waves per SIMD (157.4 -> 136.8 us a step,
// profiles/r05/wn_bwd_vec_ab.txt).
constexpr int kWnWaveX4 = 1;
// wave-per-row path: Conv1d 1x1 rows of <= 256 columns whose split sums are
// at most one round of loads per lane
__host__ __device__ inline bool wn_bwd_wave_rows(const vqx_wn_layer& l) {
  return l.kind == 0 && l.k == 1 && l.cin <= 64 * 4 * kWnWaveX4 && (l.cin / 4) * l.splits <= 64 * kWnNF;
}
// sq (optional, vqx_weight_norm_bwd_sq): every wave of block b stores the sum of
// squares of the gradient values it wrote at sq[4*b + wave] (0 if none): the
// global gradient norm's partial sums without re-reading the gradient.
__device__ __forceinline__ void wn_sq_store(float* sq, float q) {
  if (!sq) return;
  q = wave_sum(q);
  if ((threadIdx.x & 63) == 0) sq[(int64_t)blockIdx.x * (kWnThreads / 64) + (threadIdx.x >> 6)] = q;
}
__global__ __launch_bounds__(kWnThreads) void wn_bwd_kernel(const vqx_wn_layer* __restrict__ L, WnUnits U,
                                                            float* __restrict__ sq) {
  int lo = 0, hi = U.n - 1;  // the layer owning this block
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (U.off[mid] <= (int)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const vqx_wn_layer& l = L[lo];
  const int unit = (int)blockIdx.x - U.off[lo];
  if (l.kind == VQX_WN_COLREDUCE) {
    // dv[c] = sum_r v[r][c] (bias / affine gradients from per-tile partials):
    // block = kWnCrCols columns x kWnCrRG row groups, row group g summing rows
    // g, g + kWnCrRG, ... (8 loads in flight), then the groups in order
    // through LDS -- a fixed order, deterministic.
    constexpr int CC = kWnCrCols, RG = kWnThreads / kWnCrCols;
    __shared__ float crs[RG][CC];
    const int cl = threadIdx.x % CC, g = threadIdx.x / CC;
    const int c = unit * CC + cl;
    float a = 0.f;
    if (c < l.cout) {
      const float* p = l.v + c;
      int r = g;
      for (; r + 7 * RG < l.cin; r += 8 * RG) {
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = p[(int64_t)(r + u * RG) * l.cout];
#pragma unroll
        for (int u = 0; u < 8; ++u) a += t[u];
      }
      for (; r < l.cin; r += RG) a += p[(int64_t)r * l.cout];
    }
    crs[g][cl] = a;
    __syncthreads();
    float q2 = 0.f;
    if (g == 0 && c < l.cout) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < RG; ++q) t += crs[q][cl];
      l.dv[c] = t;
      q2 = t * t;
    }
    wn_sq_store(sq, q2);
    return;
  }
  if (wn_bwd_wave_rows(l)) {
    // short 1x1 rows with little split-K work (the speaker-conditioning
    // linears: 128 columns, dW written directly): one wave per row, the row's
    // sums held in registers, wave reductions only (no LDS, no barriers)
    const int o = unit * (kWnThreads / 64) + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (o >= l.cout) {
      wn_sq_store(sq, 0.f);
      return;
    }
    const int cols = l.cin, nx4 = cols / 4;
    const int64_t ss = (int64_t)l.cout * cols, srow = (int64_t)o * cols;
    const bool sbf = l.slab_dtype == VQX_BF16;
    const float* vrow = l.v + (int64_t)o * cols;
    float* dv = l.dv + (int64_t)o * cols;
    f32x4_t sm[kWnWaveX4], vv[kWnWaveX4];
    float dot = 0.f;
#pragma unroll
    for (int u = 0; u < kWnWaveX4; ++u) {
      const int x4 = lane + 64 * u;
      if (x4 < nx4) {
        vv[u] = l.g ? *(const f32x4_t*)(vrow + 4 * x4) : f32x4_t{0.f, 0.f, 0.f, 0.f};
        sm[u] = sbf ? slab_sum<true>(l.slabs, srow + 4 * x4, ss, 0, 1, l.splits)
                    : slab_sum<false>(l.slabs, srow + 4 * x4, ss, 0, 1, l.splits);
        dot = fmaf(sm[u][0], vv[u][0], fmaf(sm[u][1], vv[u][1], fmaf(sm[u][2], vv[u][2], fmaf(sm[u][3], vv[u][3], dot))));
      }
    }
    float q2 = 0.f;
    if (!l.g) {
#pragma unroll
      for (int u = 0; u < kWnWaveX4; ++u)
        if (lane + 64 * u < nx4) {
          *(f32x4_t*)(dv + 4 * (lane + 64 * u)) = sm[u];
          q2 = fmaf(sm[u][0], sm[u][0], fmaf(sm[u][1], sm[u][1], fmaf(sm[u][2], sm[u][2], fmaf(sm[u][3], sm[u][3], q2))));
        }
      wn_sq_store(sq, q2);
      return;
    }
    dot = wave_sum(dot);
    const float nrm = l.norm[o];
    const float dg = dot / nrm;
    if (lane == 0) {
      l.dg[o] = dg;
      q2 = dg * dg;
    }
    const float sc = l.g[o] / nrm, t = dg / nrm;
#pragma unroll
    for (int u = 0; u < kWnWaveX4; ++u)
      if (lane + 64 * u < nx4) {
        const f32x4_t r = {sc * (sm[u][0] - vv[u][0] * t), sc * (sm[u][1] - vv[u][1] * t),
                           sc * (sm[u][2] - vv[u][2] * t), sc * (sm[u][3] - vv[u][3] * t)};
        *(f32x4_t*)(dv + 4 * (lane + 64 * u)) = r;
        q2 = fmaf(r[0], r[0], fmaf(r[1], r[1], fmaf(r[2], r[2], fmaf(r[3], r[3], q2))));
      }
    wn_sq_store(sq, q2);
    return;
  }
  const bool rsm = l.kind == VQX_WN_RESAMPLE || l.kind == VQX_WN_RESAMPLE_T;
  const bool row_is_cout = l.kind == 0 || l.kind == VQX_WN_RESAMPLE;
  const int rows = row_is_cout ? l.cout : l.cin;
  const int o = unit;
  if (o >= rows) {
    wn_sq_store(sq, 0.f);
    return;
  }
  const int other = row_is_cout ? l.cin : l.cout;  // multiple of 4 (host-checked)
  const int K = l.k;
  const int cols = other * K;
  const int S = l.stride, SC = S * other;
  const int scols = rsm ? 3 * SC : cols;  // slab row: folded 3-tap row for the strided kinds
  __shared__ __attribute__((aligned(16))) float dw[4096];
  __shared__ float red[16];
  const int64_t slab_stride = (int64_t)rows * scols;
  const int64_t srow = (int64_t)o * scols;  // element offset of this row in split 0
  const int splits = l.splits;
  const bool sbf = l.slab_dtype == VQX_BF16;
  // the row of v, loaded before the slabs so both latencies overlap (cols <= 4096,
  // 256 threads): thread t holds the 4-element chunks c = t + 256u, 16-B loads
  // when the row is 16-B aligned (cols % 4 == 0: the data path moves a quarter
  // of the lane requests of element loads; this kernel's TD is ~90% busy)
  constexpr int kV4 = kWnVRegs / 4;
  f32x4_t vr4[kV4];
  const float* vrow = l.v + (int64_t)o * cols;
  float* dv = l.dv + (int64_t)o * cols;
  const bool al16 = ((((uintptr_t)vrow) | ((uintptr_t)dv)) & 15) == 0;
#pragma unroll
  for (int u = 0; u < kV4; ++u) {
    const int i = 4 * ((int)threadIdx.x + u * kWnThreads);
    vr4[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (l.g && i < cols) {
      if (al16) {
        vr4[u] = *(const f32x4_t*)(vrow + i);
      } else {
        vr4[u] = f32x4_t{vrow[i], vrow[i + 1], vrow[i + 2], vrow[i + 3]};
      }
    }
  }
  // Thread t sums the splits g, g+G, ... of column group x4 = t % nx4 (G = the
  // threads per group when a row has fewer than 256 groups), eight loads in
  // flight, then the G partial sums are added in g order through LDS: a fixed
  // order, so the result is deterministic.  The slab dtype is a template
  // argument of the summing loop (a dtype branch per load kept the loads from
  // being issued together).
  const int nx4 = scols / 4;
  const int G = nx4 >= (int)blockDim.x ? 1 : min(splits, (int)blockDim.x / nx4);
  const int gidx = threadIdx.x / nx4;  // split group (G == 1: every thread is group 0)
  f32x4_t* part = (f32x4_t*)dw;        // [G][nx4] partials (G > 1 only: nx4 * G <= kWnThreads -> <= 16 KiB)
  // slab column x -> dw[v index] (4 consecutive columns share the mapping)
  auto scatter = [&](int x4, const f32x4_t& sum) {
    const int x = 4 * x4;
    if (rsm) {  // slab col x = m*S*C + q*C + c -> v index c*K + S*(m-1) + q + pad (4 c's share m, q)
      const int m = x / SC, rem = x - m * SC, q = rem / other, c = rem - q * other;
      const int j = S * (m - 1) + q + l.pad;
      if (j >= 0 && j < K) {
#pragma unroll
        for (int e = 0; e < 4; ++e) dw[(c + e) * K + j] = sum[e];
      }
      return;
    }
    // slab col x = j*other + c  -> v index c*K + (kind==0 ? j : K-1-j)
    const int j = x / other, c = x - j * other;
    const int jj = l.kind == 0 ? j : K - 1 - j;
#pragma unroll
    for (int e = 0; e < 4; ++e) dw[(c + e) * K + jj] = sum[e];
  };
  const int64_t sbytes = (int64_t)splits * slab_stride * 2;
  if (G == 1 && sbf && sbytes < ((int64_t)1 << 31)) {
    // bf16 slabs: column groups x4 and x4 + 256 summed together (the 3-tap
    // rows have 384-768 groups and 4-8 splits: one pass of 8-16 loads)
    for (int x4 = threadIdx.x; x4 < nx4; x4 += 2 * kWnThreads) {
      const int x4b = x4 + kWnThreads;
      const bool hb = x4b < nx4;
      f32x4_t s0, s1;
      slab_sum2_bf(l.slabs, (int)sbytes, srow + 4 * x4, srow + 4 * (hb ? x4b : x4), slab_stride, splits, s0, s1);
      scatter(x4, s0);
      if (hb) scatter(x4b, s1);
    }
  } else {
    // G == 1: x4 = t, t + 256, ...;  G > 1: the one group x4 = t % nx4 (threads with gidx >= G idle)
    const int x4_0 = G == 1 ? (int)threadIdx.x : ((int)threadIdx.x % nx4 + (gidx < G ? 0 : nx4));
    for (int x4 = x4_0; x4 < nx4; x4 += (G == 1 ? (int)blockDim.x : nx4)) {
      const int64_t p = srow + 4 * x4;
      const int sp0 = G > 1 ? gidx : 0, step = G > 1 ? G : 1;
      const f32x4_t sum = sbf ? slab_sum<true>(l.slabs, p, slab_stride, sp0, step, splits)
                              : slab_sum<false>(l.slabs, p, slab_stride, sp0, step, splits);
      if (G > 1) part[gidx * nx4 + x4] = sum;
      else scatter(x4, sum);
    }
  }
  if (G > 1) {  // add the split groups' partials in group order, then scatter as above
    __syncthreads();
    f32x4_t sum = {0.f, 0.f, 0.f, 0.f};
    const int x4 = threadIdx.x;
    if (x4 < nx4)
      for (int g = 0; g < G; ++g) sum += part[g * nx4 + x4];
    __syncthreads();  // dw doubles as the partial buffer
    if (x4 < nx4) scatter(x4, sum);
  }
  __syncthreads();
  float q2 = 0.f;
  auto store4 = [&](int i, const f32x4_t& r) {
    if (al16) {
      *(f32x4_t*)(dv + i) = r;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) dv[i + k] = r[k];
    }
  };
  if (!l.g) {  // plain weight (weight norm removed): dv is the weight gradient itself
#pragma unroll
    for (int u = 0; u < kV4; ++u) {
      const int i = 4 * ((int)threadIdx.x + u * kWnThreads);
      if (i < cols) {
        const f32x4_t r = *(const f32x4_t*)(dw + i);
        store4(i, r);
#pragma unroll
        for (int k = 0; k < 4; ++k) q2 = fmaf(r[k], r[k], q2);
      }
    }
    wn_sq_store(sq, q2);
    return;
  }
  float dot = 0.f;
#pragma unroll
  for (int u = 0; u < kV4; ++u) {
    const int i = 4 * ((int)threadIdx.x + u * kWnThreads);
    if (i < cols) {
      const f32x4_t d4 = *(const f32x4_t*)(dw + i);
#pragma unroll
      for (int k = 0; k < 4; ++k) dot = fmaf(d4[k], vr4[u][k], dot);
    }
  }
  dot = block_sum(dot, red);
  const float nrm = l.norm[o];
  const float gg = l.g[o];
  const float dg = dot / nrm;
  if (threadIdx.x == 0) {
    l.dg[o] = dg;
    q2 = dg * dg;
  }
  const float sc = gg / nrm, t = dg / nrm;
#pragma unroll
  for (int u = 0; u < kV4; ++u) {
    const int i = 4 * ((int)threadIdx.x + u * kWnThreads);
    if (i < cols) {
      const f32x4_t d4 = *(const f32x4_t*)(dw + i);
      f32x4_t r;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        r[k] = sc * (d4[k] - vr4[u][k] * t);
        q2 = fmaf(r[k], r[k], q2);
      }
      store4(i, r);
    }
  }
  wn_sq_store(sq, q2);
}

// --------------------------------------------------------------- groupnorm
// Partial moments per (b, g, part): two-pass within the part (mean, then
// centred sum of squares), combined with Chan's formula in finalize.
constexpr int kGnParts = 8;
constexpr int kGnBwdParts = 32;  // row parts of the GroupNorm-backward reduction

template <typename T>
__global__ __launch_bounds__(256) void gn_partial_kernel(const T* __restrict__ x, int ldx, int T_, int C, int G,
                                                         float* __restrict__ part) {
  const int p = blockIdx.x, bg = blockIdx.y;
  const int b = bg / G, g = bg - b * G;
  const int cg = C / G;
  const int r0 = p * T_ / kGnParts, r1 = (p + 1) * T_ / kGnParts;
  const int64_t nrows = r1 - r0;
  const int64_t cnt = nrows * cg;
  __shared__ float red[16];
  const T* base = x + ((int64_t)b * T_ + r0) * ldx + g * cg;
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < cnt; i += blockDim.x) {
    const int64_t rr = i / cg, cc = i - rr * cg;
    s += Elem<T>::ld(base, rr * ldx + cc);
  }
  s = block_sum(s, red);
  const float mean = cnt ? s / (float)cnt : 0.f;
  float m2 = 0.f;
  for (int64_t i = threadIdx.x; i < cnt; i += blockDim.x) {
    const int64_t rr = i / cg, cc = i - rr * cg;
    const float d = Elem<T>::ld(base, rr * ldx + cc) - mean;
    m2 = fmaf(d, d, m2);
  }
  m2 = block_sum(m2, red);
  if (threadIdx.x == 0) {
    float* o = part + ((int64_t)bg * kGnParts + p) * 3;
    o[0] = (float)cnt;
    o[1] = mean;
    o[2] = m2;
  }
}

__global__ void gn_finalize_kernel(const float* __restrict__ part, int nbg, float eps, float* __restrict__ mr) {
  const int bg = blockIdx.x * blockDim.x + threadIdx.x;
  if (bg >= nbg) return;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  for (int p = 0; p < kGnParts; ++p) {
    const float* o = part + ((int64_t)bg * kGnParts + p) * 3;
    const double nb = o[0];
    if (nb == 0.0) continue;
    const double d = (double)o[1] - mean;
    const double nn = n + nb;
    mean += d * nb / nn;
    m2 += (double)o[2] + d * d * n * nb / nn;
    n = nn;
  }
  const float var = n > 0.0 ? (float)(m2 / n) : 0.f;
  mr[2 * bg] = (float)mean;
  mr[2 * bg + 1] = 1.0f / sqrtf(var + eps);
}

// Combine the GEMM GNSTATS tiles [N/128][ntn][4] = (count, mean, M2, -) of
// utterance b's row groups and group g's column tiles (double, fixed order).
__global__ void gn_finalize_tiles_kernel(const float* __restrict__ part, int B, int G, int rg_per_utt, int ntn,
                                         int tn_per_group, float eps, float* __restrict__ mr) {
  const int bg = blockIdx.x * blockDim.x + threadIdx.x;
  if (bg >= B * G) return;
  const int b = bg / G, g = bg - b * G;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  for (int r = 0; r < rg_per_utt; ++r)
    for (int t = 0; t < tn_per_group; ++t) {
      const float* o = part + ((int64_t)(b * rg_per_utt + r) * ntn + g * tn_per_group + t) * 4;
      const double nb = o[0];
      if (nb == 0.0) continue;
      const double d = (double)o[1] - mean;
      const double nn = n + nb;
      mean += d * nb / nn;
      m2 += (double)o[2] + d * d * n * nb / nn;
      n = nn;
    }
  const float var = n > 0.0 ? (float)(m2 / n) : 0.f;
  mr[2 * bg] = (float)mean;
  mr[2 * bg + 1] = 1.0f / sqrtf(var + eps);
}


// ---- 16-byte chunk helpers (8 bf16 or 4 f32 per chunk) -------------------
template <typename T> struct Vec;
template <> struct Vec<bf16_t> {
  static constexpr int N = 8;
  typedef uint4 raw_t;  // the 16-B chunk as loaded (cvt: to floats where they are used)
  __device__ static __forceinline__ raw_t ld(const bf16_t* p) { return *(const uint4*)p; }
  __device__ static __forceinline__ void cvt(const raw_t& u, float* f) {
    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { f[2 * i] = __uint_as_float(w[i] << 16); f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
  }
  __device__ static __forceinline__ void load(const bf16_t* p, float* f) { cvt(ld(p), f); }
  __device__ static __forceinline__ void store(bf16_t* p, const float* f) {
    unsigned w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
    *(uint4*)p = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <> struct Vec<float> {
  static constexpr int N = 4;
  typedef f32x4_t raw_t;
  __device__ static __forceinline__ raw_t ld(const float* p) { return *(const f32x4_t*)p; }
  __device__ static __forceinline__ void cvt(const raw_t& v, float* f) { f[0] = v[0]; f[1] = v[1]; f[2] = v[2]; f[3] = v[3]; }
  __device__ static __forceinline__ void load(const float* p, float* f) { cvt(ld(p), f); }
  __device__ static __forceinline__ void store(float* p, const float* f) {
    f32x4_t v = {f[0], f[1], f[2], f[3]};
    *(f32x4_t*)p = v;
  }
};

// GroupNorm partial moments, vectorised: block (part p, utterance-group bg);
// thread = (chunk of the group's columns, row group).  Requires the group's
// chunk count cpr to divide 256.
template <typename T>
__global__ __launch_bounds__(256) void gn_partial_vec_kernel(const T* __restrict__ x, int ldx, int T_, int C, int G,
                                                             int cpr, float* __restrict__ part) {
  constexpr int V = Vec<T>::N;
  const int p = blockIdx.x, bg = blockIdx.y;
  const int b = bg / G, g = bg - b * G;
  const int cg = C / G;
  const int r0 = p * T_ / kGnParts, r1 = (p + 1) * T_ / kGnParts;
  const int ch = threadIdx.x % cpr, rg = threadIdx.x / cpr, nrg = 256 / cpr;
  __shared__ float red[16];
  const T* base = x + ((int64_t)b * T_) * ldx + g * cg + ch * V;
  float s = 0.f;
  for (int r = r0 + rg; r < r1; r += nrg) {
    float f[V];
    Vec<T>::load(base + (int64_t)r * ldx, f);
#pragma unroll
    for (int i = 0; i < V; ++i) s += f[i];
  }
  s = block_sum(s, red);
  const int64_t cnt = (int64_t)(r1 - r0) * cg;
  const float mean = cnt ? s / (float)cnt : 0.f;
  float m2 = 0.f;
  for (int r = r0 + rg; r < r1; r += nrg) {
    float f[V];
    Vec<T>::load(base + (int64_t)r * ldx, f);
#pragma unroll
    for (int i = 0; i < V; ++i) { const float d = f[i] - mean; m2 = fmaf(d, d, m2); }
  }
  m2 = block_sum(m2, red);
  if (threadIdx.x == 0) {
    float* o = part + ((int64_t)bg * kGnParts + p) * 3;
    o[0] = (float)cnt;
    o[1] = mean;
    o[2] = m2;
  }
}

// Gradient w.r.t. the GroupNorm output h for a chunk of V channels.
//   glu: channels [c, c+V) of the tanh half AND [c+half, c+half+V) of the
//        sigmoid half (dy = dL/dg has `half` columns);
//   else: channels [c, c+V) (dy = dL/dh), single group set by the caller.
template <typename T>
__device__ __forceinline__ void gn_dh_chunk(const T* dy, int lddy, const T* u, int ldu, int64_t n, int c, int half,
                                            bool glu, const float* mr4, const float* gamma, const float* beta,
                                            float* dha, float* xa, float* dhb, float* xb) {
  constexpr int V = Vec<T>::N;
  float g[V], ua[V];
  Vec<T>::load(dy + n * lddy + c, g);
  Vec<T>::load(u + n * ldu + c, ua);
  if (!glu) {
#pragma unroll
    for (int i = 0; i < V; ++i) { dha[i] = g[i]; xa[i] = (ua[i] - mr4[0]) * mr4[1]; }
    return;
  }
  float ub[V];
  Vec<T>::load(u + n * ldu + c + half, ub);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const float xha = (ua[i] - mr4[0]) * mr4[1];
    const float xhb = (ub[i] - mr4[2]) * mr4[3];
    const float ha = xha * gamma[c + i] + beta[c + i];
    const float hb = xhb * gamma[c + half + i] + beta[c + half + i];
    const float ta = ftanh<sizeof(T) == 2>(ha);
    const float sb = fsigmoid<sizeof(T) == 2>(hb);
    dha[i] = g[i] * sb * (1.f - ta * ta);
    dhb[i] = g[i] * ta * (sb * (1.f - sb));
    xa[i] = xha;
    xb[i] = xhb;
  }
}

// pass 1 (vectorised): per (utterance, part) S1_g = sum gamma*dh, S2_g = sum gamma*dh*xhat
template <typename T>
__global__ __launch_bounds__(256) void gn_bwd_reduce_vec_kernel(const T* __restrict__ dy, int lddy,
                                                                const T* __restrict__ u, int ldu, int T_, int C, int G,
                                                                int glu, int cpr, const float* __restrict__ mr,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta,
                                                                float* __restrict__ part) {
  constexpr int V = Vec<T>::N;
  const int p = blockIdx.x, b = blockIdx.y;
  const int r0 = p * T_ / kGnBwdParts, r1 = (p + 1) * T_ / kGnBwdParts;
  const int ch = threadIdx.x % cpr, rg = threadIdx.x / cpr, nrg = 256 / cpr;
  const int half = C / 2;
  const int c = ch * V;
  const float* mr4 = mr + (int64_t)b * G * 2;
  __shared__ float red[16];
  float s1a = 0.f, s2a = 0.f, s1b = 0.f, s2b = 0.f;
  for (int r = r0 + rg; r < r1; r += nrg) {
    const int64_t n = (int64_t)b * T_ + r;
    float dha[V], xa[V], dhb[V], xb[V];
    gn_dh_chunk<T>(dy, lddy, u, ldu, n, c, half, glu, mr4, gamma, beta, dha, xa, dhb, xb);
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const float ga = gamma[c + i] * dha[i];
      s1a += ga;
      s2a = fmaf(ga, xa[i], s2a);
      if (glu) {
        const float gb = gamma[c + half + i] * dhb[i];
        s1b += gb;
        s2b = fmaf(gb, xb[i], s2b);
      }
    }
  }
  s1a = block_sum(s1a, red);
  __syncthreads();
  s2a = block_sum(s2a, red);
  __syncthreads();
  if (glu) {
    s1b = block_sum(s1b, red);
    __syncthreads();
    s2b = block_sum(s2b, red);
  }
  if (threadIdx.x == 0) {
    float* o = part + ((int64_t)b * kGnBwdParts + p) * G * 2;
    o[0] = s1a;
    o[1] = s2a;
    if (glu) { o[2] = s1b; o[3] = s2b; }
  }
}

// pass 2 (vectorised): du and per-(utterance, channel) sums of du (bias /
// conv_cond gradients), dh*xhat (dgamma) and dh (dbeta).  Block = one
// utterance x 64 channels x all T rows, so the per-utterance sums are complete
// inside the block (deterministic, no atomics).  A thread owns 4 channels
// (8-B bf16 / 16-B fp32 accesses; 16 lanes cover a 64-channel row segment)
// in one of 32 row groups and loads two rows before the math of either: the
// kernel is bound by the loads in flight per CU, and 4 channels a thread keep
// it at ~100 VGPRs (8 channels: 176, two waves per SIMD).
#ifndef VQX_GN_NR  // rows in flight per thread in gn_bwd_apply_vec_kernel
#define VQX_GN_NR 2
#endif
constexpr int kGnApplyRG = 32, kGnApplyW = 4, kGnApplyNR = VQX_GN_NR;
template <typename T> struct Vec4;
template <> struct Vec4<bf16_t> {
  typedef uint2 raw_t;
  __device__ static __forceinline__ raw_t ld(const bf16_t* p) { return *(const uint2*)p; }
  __device__ static __forceinline__ void cvt(const raw_t& u, float* f) {
    f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
    f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
  }
  __device__ static __forceinline__ void load(const bf16_t* p, float* f) { cvt(ld(p), f); }
  __device__ static __forceinline__ void store(bf16_t* p, const float* f) {
    *(uint2*)p = make_uint2(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]));
  }
};
template <> struct Vec4<float> : Vec<float> {};
template <typename T, bool GLU>
__global__ __launch_bounds__(512) void gn_bwd_apply_vec_kernel(const T* __restrict__ dy, int lddy,
                                                               const T* __restrict__ u, int ldu, T* __restrict__ du,
                                                               int lddu, int T_, int C, int G, int, int cpr,
                                                               const float* __restrict__ mr,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta,
                                                               const float* __restrict__ part, int nparts,
                                                               int pstride, float* __restrict__ colsum_b,
                                                               float* __restrict__ dgamma_b, float* __restrict__ dbeta_b) {
  constexpr bool glu = GLU;
  constexpr int W = kGnApplyW, RG = kGnApplyRG;
  const int cpw = cpr * (Vec<T>::N / W);  // W-channel chunks per half row
  const int b = blockIdx.y;
  const int ch = blockIdx.x * 16 + (threadIdx.x & 15), rg = threadIdx.x >> 4;
  const bool active = ch < cpw;
  const int half = C / 2;
  const int c = ch * W;
  const float* mr4 = mr + (int64_t)b * G * 2;
  const int ng = glu ? 2 : 1;
  const int lane = threadIdx.x & 63;
  // The utterance's partials, one part per lane (nparts <= 64), loaded first,
  // then gamma / beta and the first two rows as raw chunks; every wave then
  // sums the partials in part order through shuffles (no LDS, no barrier), so
  // the sum waits on the partial loads only and runs under the rows' flight.
  // (The LDS-staged sum ran before any row load was issued.)
  const bool shfl_sum = nparts <= 64;
  float q0 = 0.f, q1 = 0.f, q2 = 0.f, q3 = 0.f;
  if (shfl_sum && lane < nparts) {
    const float* o = part + ((int64_t)b * nparts + lane) * pstride;
    q0 = o[0];
    q1 = o[1];
    if (glu) { q2 = o[2]; q3 = o[3]; }
  }
  float ga[W], ba[W], gb[W], bb[W];
  const int cc = active ? c : 0;  // inactive lanes load chunk 0 and discard it (no branch to join)
#pragma unroll
  for (int i = 0; i < W; ++i) {
    ga[i] = gamma[cc + i];
    ba[i] = beta[cc + i];
    gb[i] = glu ? gamma[cc + half + i] : 0.f;
    bb[i] = glu ? beta[cc + half + i] : 0.f;
  }
  // the first NR rows as raw chunks (rows clamped into the utterance), converted after the sums
  typedef typename Vec4<T>::raw_t raw_t;
  constexpr int NR = kGnApplyNR;
  const int64_t nb0 = (int64_t)b * T_;
  raw_t pg[NR], pa[NR], pb[NR];
  auto load_rows = [&](int r) {
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int64_t nc = nb0 + min(r + k * RG, T_ - 1);
      pg[k] = Vec4<T>::ld(dy + nc * lddy + cc);
      pa[k] = Vec4<T>::ld(u + nc * ldu + cc);
      pb[k] = glu ? Vec4<T>::ld(u + nc * ldu + cc + half) : raw_t{};
    }
  };
  load_rows(rg);
  float m1a = 0.f, m2a = 0.f, m1b = 0.f, m2b = 0.f;
  {
    const int cg = C / G;
    const float M = (float)T_ * (float)cg;
    float S1a = 0.f, S2a = 0.f, S1b = 0.f, S2b = 0.f;
    // two loops: a global load inside the shuffle loop would make every
    // iteration wait on all loads in flight
    if (shfl_sum) {
      for (int q = 0; q < nparts; ++q) {
        S1a += __shfl(q0, q, 64);
        S2a += __shfl(q1, q, 64);
        if (glu) { S1b += __shfl(q2, q, 64); S2b += __shfl(q3, q, 64); }
      }
    } else {
      for (int q = 0; q < nparts; ++q) {
        const float* o = part + ((int64_t)b * nparts + q) * pstride;
        S1a += o[0];
        S2a += o[1];
        if (glu) { S1b += o[2]; S2b += o[3]; }
      }
    }
    m1a = S1a / M; m2a = S2a / M; m1b = S1b / M; m2b = S2b / M;
  }
  float a_du[2][W], a_dg[2][W], a_db[2][W];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < W; ++i) { a_du[s][i] = 0.f; a_dg[s][i] = 0.f; a_db[s][i] = 0.f; }
  auto row = [&](int64_t n, const float* g, const float* ua, const float* ub) {
    float dha[W], xa[W], dhb[W], xb[W], oa[W];
    gn_row_math<T, W>(g, ua, ub, glu, mr4, ga, ba, gb, bb, dha, xa, dhb, xb);
    gn_dx<W>(dha, xa, ga, mr4[1], m1a, m2a, oa);
#pragma unroll
    for (int i = 0; i < W; ++i) {
      a_du[0][i] += oa[i];
      a_dg[0][i] = fmaf(dha[i], xa[i], a_dg[0][i]);
      a_db[0][i] += dha[i];
    }
    Vec4<T>::store(du + n * lddu + c, oa);
    if (glu) {
      float ob[W];
      gn_dx<W>(dhb, xb, gb, mr4[3], m1b, m2b, ob);
#pragma unroll
      for (int i = 0; i < W; ++i) {
        a_du[1][i] += ob[i];
        a_dg[1][i] = fmaf(dhb[i], xb[i], a_dg[1][i]);
        a_db[1][i] += dhb[i];
      }
      Vec4<T>::store(du + n * lddu + c + half, ob);
    }
  };
  if (active) {
    // NR rows in flight, processed in row order (the column sums' order does
    // not depend on NR)
    for (int r = rg; r < T_; r += NR * RG) {
      if (r != rg) load_rows(r);
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        if (r + k * RG < T_) {
          float g0[W], ua0[W], ub0[W];
          Vec4<T>::cvt(pg[k], g0);
          Vec4<T>::cvt(pa[k], ua0);
          if (glu) Vec4<T>::cvt(pb[k], ub0);
          row(nb0 + r + k * RG, g0, ua0, ub0);
        }
      }
    }
  }
  __shared__ float lds[RG][16][2 * W];
  auto dump = [&](const float (&a)[2][W], float* out) {
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < W; ++i) lds[rg][threadIdx.x & 15][s * W + i] = a[s][i];
    __syncthreads();
    // 128 threads finish 16 chunks x 2 halves x W columns
    for (int e = threadIdx.x; e < 16 * 2 * W; e += 512) {
      const int cl = e / (2 * W), rem = e - cl * 2 * W, s = rem / W, i = rem - s * W;
      const int chg = blockIdx.x * 16 + cl;
      if (chg >= cpw || s >= ng || !out) continue;
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < RG; ++q) t += lds[q][cl][rem];
      out[(int64_t)b * C + chg * W + s * half + i] = t;
    }
  };
  dump(a_du, colsum_b);
  dump(a_dg, dgamma_b);
  dump(a_db, dbeta_b);
}


// g = tanh(GN(u)[:, :half]) * sigmoid(GN(u)[:, half:]), GroupNorm with G=2,
// one 16-B chunk of V channels per thread (layers.py:236-242).
template <typename T>
__global__ __launch_bounds__(256) void gn_glu_fwd_vec_kernel(const T* __restrict__ u, int ldu, T* __restrict__ g,
                                                             int ldg, int n_rows, int T_, int half, int cpr,
                                                             const float* __restrict__ mr,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta,
                                                             const float* __restrict__ tiles, float eps,
                                                             float* __restrict__ mr_out, int fpb) {
  // block = fpb frames; thread = (chunk, row slot); cpr divides 256
  constexpr int V = Vec<T>::N;
  const int ch = threadIdx.x % cpr, rs = threadIdx.x / cpr, nrs = 256 / cpr;
  const int c = ch * V;
  const int lane = threadIdx.x & 63;
  // In-launch statistics (tiles != null): this block's utterance (T % fpb == 0:
  // the fpb frames share one) merged from the producing GEMM's GNSTATS tiles,
  // as gn_finalize_tiles_kernel does, by wave 0: lane k loads tile k (group
  // k / nt), then the tiles are merged in order through shuffles, lane parity
  // choosing the group, in double, and lanes 0 / 1 leave the result in LDS
  // for the barrier.  The tile loads go out first, then gamma / beta and the
  // first rows as raw chunks: the merge waits on the tile loads only (vmcnt
  // counts in issue order) and the barrier (an LDS wait on gfx950) on the
  // merge, with the rows in flight.  (Round 5: with the rows loaded after the
  // barrier, as program order had them, the merge cost 2.6 us of a 13.2 us
  // launch against the precomputed-statistics path; loads converted as they
  // are issued would wait right there.  The merge in every wave, without the
  // barrier, cost as much in f64 issue as it saved.)
  const int b0 = blockIdx.x * fpb / T_, rg = T_ / 128, ntn = 2 * half / 128, tpg = ntn / 2, nt = rg * tpg;
  const bool shfl_merge = 2 * nt <= 64;  // every tile in one lane
  float tl0 = 0.f, tl1 = 0.f, tl2 = 0.f;
  if (tiles && shfl_merge && (int)threadIdx.x < 2 * nt) {
    const int gi = lane / nt, k = lane - gi * nt, r = k / tpg, t = k - r * tpg;
    const float* o = tiles + ((int64_t)(b0 * rg + r) * ntn + gi * tpg + t) * 4;
    tl0 = o[0];
    tl1 = o[1];
    tl2 = o[2];
  }
  float ga[V], ba[V], gb[V], bb[V];
#pragma unroll
  for (int i = 0; i < V; ++i) { ga[i] = gamma[c + i]; ba[i] = beta[c + i]; gb[i] = gamma[c + half + i]; bb[i] = beta[c + half + i]; }
  // two rows' loads in flight before the math of either; the first pair's
  // raw chunks are converted after the merge, so it does not wait on them
  typedef typename Vec<T>::raw_t raw_t;
  const int rend = min(n_rows, blockIdx.x * fpb + fpb);
  int r = blockIdx.x * fpb + rs;
  const bool pair = r + nrs < rend, one = r < rend;
  // clamped rows (every block holds at least one): the loads need no branch,
  // whose join would wait on them
  const int r0c = one ? r : rend - 1, r1c = pair ? r + nrs : r0c;
  const raw_t qa0 = Vec<T>::ld(u + (int64_t)r0c * ldu + c), qb0 = Vec<T>::ld(u + (int64_t)r0c * ldu + c + half);
  const raw_t qa1 = Vec<T>::ld(u + (int64_t)r1c * ldu + c), qb1 = Vec<T>::ld(u + (int64_t)r1c * ldu + c + half);
  float s_ma = 0.f, s_ra = 0.f, s_mb = 0.f, s_rb = 0.f;  // mean / rstd of groups a and b (tiles path)
  __shared__ float smr[4];
  if (tiles && threadIdx.x < 64) {
    const int gi = lane & 1;
    double n = 0.0, mean = 0.0, m2 = 0.0;
    auto merge = [&](float o0, float o1, float o2) {
      const double nb = o0;
      if (nb == 0.0) return;
      const double d = (double)o1 - mean;
      const double nn = n + nb;
      mean += d * nb / nn;
      m2 += (double)o2 + d * d * n * nb / nn;
      n = nn;
    };
    // two loops: a global load inside the shuffle loop would make every
    // iteration wait on all loads in flight
    if (shfl_merge) {
      for (int k = 0; k < nt; ++k) {
        const int src = gi * nt + k;
        merge(__shfl(tl0, src, 64), __shfl(tl1, src, 64), __shfl(tl2, src, 64));
      }
    } else {
      for (int rr = 0; rr < rg; ++rr)
        for (int t = 0; t < tpg; ++t) {
          const float* o = tiles + ((int64_t)(b0 * rg + rr) * ntn + gi * tpg + t) * 4;
          merge(o[0], o[1], o[2]);
        }
    }
    const float var = n > 0.0 ? (float)(m2 / n) : 0.f;
    const float mf = (float)mean, rf = 1.0f / sqrtf(var + eps);
    if (threadIdx.x < 2) {
      smr[2 * gi] = mf;
      smr[2 * gi + 1] = rf;
      if ((blockIdx.x * fpb) % T_ == 0) {  // the utterance's first block stores them
        mr_out[4 * b0 + 2 * gi] = mf;
        mr_out[4 * b0 + 2 * gi + 1] = rf;
      }
    }
  }
  if (tiles) {
    __syncthreads();  // (waits on LDS only: the rows' loads stay in flight)
    s_ma = smr[0];
    s_ra = smr[1];
    s_mb = smr[2];
    s_rb = smr[3];
  }
  auto row = [&](int r, const float* ua, const float* ub) {
    const int b = r / T_;
    float ma, ra, mb, rb;
    if (tiles) { ma = s_ma; ra = s_ra; mb = s_mb; rb = s_rb; }
    else { ma = mr[4 * b + 0]; ra = mr[4 * b + 1]; mb = mr[4 * b + 2]; rb = mr[4 * b + 3]; }
    float o[V];
#pragma unroll
    for (int i = 0; i < V; ++i)
      o[i] = ftanh<sizeof(T) == 2>((ua[i] - ma) * ra * ga[i] + ba[i]) *
             fsigmoid<sizeof(T) == 2>((ub[i] - mb) * rb * gb[i] + bb[i]);
    Vec<T>::store(g + (int64_t)r * ldg + c, o);
  };
  if (!one) return;
  float ua0[V], ub0[V], ua1[V], ub1[V];
  Vec<T>::cvt(qa0, ua0);
  Vec<T>::cvt(qb0, ub0);
  row(r, ua0, ub0);
  if (!pair) return;
  Vec<T>::cvt(qa1, ua1);
  Vec<T>::cvt(qb1, ub1);
  row(r + nrs, ua1, ub1);
  for (r += 2 * nrs; r + nrs < rend; r += 2 * nrs) {
    Vec<T>::load(u + (int64_t)r * ldu + c, ua0);
    Vec<T>::load(u + (int64_t)r * ldu + c + half, ub0);
    Vec<T>::load(u + (int64_t)(r + nrs) * ldu + c, ua1);
    Vec<T>::load(u + (int64_t)(r + nrs) * ldu + c + half, ub1);
    row(r, ua0, ub0);
    row(r + nrs, ua1, ub1);
  }
  if (r < rend) {
    Vec<T>::load(u + (int64_t)r * ldu + c, ua0);
    Vec<T>::load(u + (int64_t)r * ldu + c + half, ub0);
    row(r, ua0, ub0);
  }
}

// g = LeakyReLU_0.2(GroupNorm_{G=1}(h)): the LeakyReLU heading each further
// conv of a residual stack with stack_layers > 1 (layers.py:156-161), one
// 16-B chunk of V channels per thread.
template <typename T>
__global__ __launch_bounds__(256) void gn_lrelu_fwd_kernel(const T* __restrict__ h, int ldh, T* __restrict__ g, int ldg,
                                                           int64_t n_rows, int T_, int cpr,
                                                           const float* __restrict__ mr,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta) {
  constexpr int V = Vec<T>::N;
  const int64_t total = n_rows * cpr;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / cpr;
    const int c = (int)(i - r * cpr) * V;
    const int b = (int)(r / T_);
    const float m = mr[2 * b], rs = mr[2 * b + 1];
    float x[V];
    Vec<T>::load(h + r * ldh + c, x);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float v = (x[k] - m) * rs * gamma[c + k] + beta[c + k];
      x[k] = v > 0.f ? v : 0.2f * v;
    }
    Vec<T>::store(g + r * ldg + c, x);
  }
}

// single-pass column sums for short inputs (rows <= ~2048): 64 columns x 4 row groups per block
template <typename T>
__global__ __launch_bounds__(256) void colsum_small_kernel(const T* __restrict__ x, int ldx, int64_t n_rows, int C,
                                                           float* __restrict__ out, int accum) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  __shared__ float acc[4][64];
  float s = 0.f;
  if (c < C)
    for (int64_t r = rg; r < n_rows; r += 4) s += Elem<T>::ld(x, r * ldx + c);
  acc[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && c < C) {
    const int l = threadIdx.x & 63;
    const float t = acc[0][l] + acc[1][l] + acc[2][l] + acc[3][l];
    out[c] = accum ? out[c] + t : t;
  }
}

// vectorised partial column sums: 32 chunks x 8 row groups per block
template <typename T>
// Lanes [0, L) of each row group cover L column chunks of V; 256/L row groups
// stride the rows, so narrow outputs (bias gradients of 64..128 columns) keep
// every lane of the block busy instead of 10 of 32.
__global__ __launch_bounds__(256) void colsum_partial_vec_kernel(const T* __restrict__ x, int ldx, int64_t n_rows,
                                                                 int C, int nparts, int L, float* __restrict__ part) {
  constexpr int V = Vec<T>::N;
  const int lane = threadIdx.x % L;
  const int rg = threadIdx.x / L, R = 256 / L;
  const int chunk = blockIdx.x * L + lane;
  const int p = blockIdx.y;
  const int64_t r0 = n_rows * p / nparts, r1 = n_rows * (p + 1) / nparts;
  const int c = chunk * V;
  float s[V];
#pragma unroll
  for (int i = 0; i < V; ++i) s[i] = 0.f;
  if (c < C)
#pragma unroll 4
    for (int64_t r = r0 + rg; r < r1; r += R) {
      float f[V];
      Vec<T>::load(x + r * ldx + c, f);
#pragma unroll
      for (int i = 0; i < V; ++i) s[i] += f[i];
    }
  __shared__ float lds[256 * V];
#pragma unroll
  for (int i = 0; i < V; ++i) lds[threadIdx.x * V + i] = s[i];
  __syncthreads();
  for (int e = threadIdx.x; e < L * V; e += 256) {
    const int cc = blockIdx.x * L * V + e;
    if (cc < C) {
      float t = 0.f;
      for (int q = 0; q < R; ++q) t += lds[q * L * V + e];
      part[(int64_t)p * C + cc] = t;
    }
  }
}

// ------------------------------------------------------------------ colsum
template <typename T>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const T* __restrict__ x, int ldx, int64_t n_rows, int C,
                                                             int nparts, float* __restrict__ part) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const int p = blockIdx.y;
  const int64_t r0 = n_rows * p / nparts, r1 = n_rows * (p + 1) / nparts;
  __shared__ float acc[4][64];
  float s = 0.f;
  if (c < C)
    for (int64_t r = r0 + rg; r < r1; r += 4) s += Elem<T>::ld(x, r * ldx + c);
  acc[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && c < C) {
    const int l = threadIdx.x & 63;
    part[(int64_t)p * C + c] = acc[0][l] + acc[1][l] + acc[2][l] + acc[3][l];
  }
}

// One wave per column: lanes stride the (<= 64) partials, then a fixed-order
// butterfly, so the result is deterministic and no lane walks 64 loads.
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part, int nparts, int C,
                                                           float* __restrict__ out, int accum) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= C) return;
  float s = 0.f;
  for (int p = lane; p < nparts; p += 64) s += part[(int64_t)p * C + c];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) out[c] = accum ? out[c] + s : s;
}

// ------------------------------------------------------------------ layout
// one 32 x 32 tile (bx over T, by over C, b the batch row); tile: LDS
template <typename T>
__device__ __forceinline__ void nct_to_ntc_tile(const float* __restrict__ x, int C, int T_, T* __restrict__ y, int ldy,
                                                int bx, int by, int b, float (*tile)[33]) {
  const int t0 = bx * 32, c0 = by * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 rows per pass
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, t = t0 + tx;
    tile[i][tx] = (c < C && t < T_) ? x[((int64_t)b * C + c) * T_ + t] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int t = t0 + i, c = c0 + tx;
    if (c < C && t < T_) Elem<T>::st(y, ((int64_t)b * T_ + t) * ldy + c, tile[tx][i]);
  }
}
template <typename T>
__global__ void nct_to_ntc_kernel(const float* __restrict__ x, int B, int C, int T_, T* __restrict__ y, int ldy) {
  __shared__ float tile[32][33];
  nct_to_ntc_tile<T>(x, C, T_, y, ldy, blockIdx.x, blockIdx.y, blockIdx.z, tile);
}

template <typename T>
__global__ void ntc_to_nct_kernel(const T* __restrict__ y, int ldy, int B, int C, int T_, float* __restrict__ x) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z;
  const int t0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int t = t0 + i, c = c0 + tx;
    tile[i][tx] = (c < C && t < T_) ? Elem<T>::ld(y, ((int64_t)b * T_ + t) * ldy + c) : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, t = t0 + tx;
    if (c < C && t < T_) x[((int64_t)b * C + c) * T_ + t] = tile[tx][i];
  }
}

// ----------------------------------------------------------------- logloss
template <typename T>
__global__ __launch_bounds__(256) void logloss_kernel(const float* __restrict__ x, const float* __restrict__ xh, int ldxh,
                                                      int B, int C, int T_, float gscale, T* __restrict__ dx, int lddx,
                                                      float* __restrict__ part) {
  __shared__ float red[16];
  const int64_t total = (int64_t)B * T_ * C;
  float s = 0.f;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)e / C;  // 32-bit: total < 2^31 (host-checked)
    const int c = (int)e - n * C;
    const int b = (int)n / T_, t = (int)n - b * T_;
    const float xv = x[((int64_t)b * C + c) * T_ + t];
    const float d = xh[(int64_t)n * ldxh + c] - xv;
    s += 0.5f * (kLog2Pi + d * d);
    if (dx) Elem<T>::st(dx, (int64_t)n * lddx + c, d * gscale);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// The same over (utterance, 64-frame tile) blocks: the tile of x (C channels
// x 64 frames, NCT) is read row by row (coalesced) into LDS, then xhat (f32)
// and dx move as whole 4-channel chunks of their frame-major rows (C % 4 ==
// 0), each chunk's channels taken from the LDS tile.  (The flat kernel above
// reads x with a stride of T floats between neighbouring lanes.)
constexpr int kLlTile = 64;
template <typename T>
__global__ __launch_bounds__(256) void logloss_tile_kernel(const float* __restrict__ x, const float* __restrict__ xh,
                                                           int ldxh, int C, int T_, float gscale, T* __restrict__ dx,
                                                           int lddx, float* __restrict__ part) {
  extern __shared__ float xs[];  // [C][kLlTile + 1]
  __shared__ float red[16];
  const int b = blockIdx.y, t0 = blockIdx.x * kLlTile;
  const int nt = min(kLlTile, T_ - t0);
  const float* xb = x + (int64_t)b * C * T_ + t0;
  // loads batched U at a time (clamped addresses, no branch), then their LDS writes:
  // a load-store pair per element paid one memory latency each
  constexpr int U = 16;
  for (int e0 = threadIdx.x; e0 < C * kLlTile; e0 += 256 * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = min(e0 + 256 * u, C * kLlTile - 1), c = e / kLlTile, t = min(e - c * kLlTile, nt - 1);
      v[u] = xb[(int64_t)c * T_ + t];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + 256 * u, c = e / kLlTile, t = e - c * kLlTile;
      if (e < C * kLlTile) xs[c * (kLlTile + 1) + t] = t < nt ? v[u] : 0.f;
    }
  }
  __syncthreads();
  const int cpr = C / 4;  // chunks per frame row
  const int64_t n0 = (int64_t)b * T_ + t0;
  const int nq = nt * cpr;
  float s = 0.f;
  constexpr int U2 = 8;
  for (int q0 = threadIdx.x; q0 < nq; q0 += 256 * U2) {
    f32x4_t h[U2];
#pragma unroll
    for (int u = 0; u < U2; ++u) {
      const int qq = min(q0 + 256 * u, nq - 1), t = qq / cpr, c0 = (qq - t * cpr) * 4;
      h[u] = *(const f32x4_t*)(xh + (n0 + t) * ldxh + c0);
    }
#pragma unroll
    for (int u = 0; u < U2; ++u) {
      const int q = q0 + 256 * u;
      if (q >= nq) break;
      const int t = q / cpr, c0 = (q - t * cpr) * 4;
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d = h[u][k] - xs[(c0 + k) * (kLlTile + 1) + t];
        s += 0.5f * (kLog2Pi + d * d);
        o[k] = d * gscale;
      }
      if (dx) Vec4<T>::store(dx + (n0 + t) * lddx + c0, o);
    }
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.y * gridDim.x + blockIdx.x] = s;
}

__global__ void sum_partials_scale_kernel(const float* __restrict__ p, int n, float scale, float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += p[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[0] = s * scale;
}

// two such sums in one launch (the log-loss total and another partial set, e.g.
// the VQ kernel's commitment partials): each as sum_partials_scale_kernel sums it
__global__ void sum_partials2_kernel(const float* __restrict__ p, int n, float scale, float* __restrict__ out,
                                     const float* __restrict__ p2, int n2, float scale2, float* __restrict__ out2) {
  __shared__ float red[2][16];
  float v[2] = {0.f, 0.f};
  for (int i = threadIdx.x; i < n; i += blockDim.x) v[0] += p[i];
  for (int i = threadIdx.x; i < n2; i += blockDim.x) v[1] += p2[i];
  block_sum_n<2>(v, red);
  if (threadIdx.x == 0) {
    out[0] = v[0] * scale;
    out2[0] = v[1] * scale2;
  }
}

// ------------------------------------------------------------ small kernels
template <typename T>
__global__ void time_gather_kernel(const T* __restrict__ x, T* __restrict__ y, int B, int T_, int C,
                                   const int* __restrict__ src) {
  const int64_t total = (int64_t)B * T_ * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)e / C;  // 32-bit: total < 2^31 (host-checked)
    const int c = (int)e - n * C;
    const int b = (int)n / T_, t = (int)n - b * T_;
    y[e] = x[((int64_t)b * T_ + src[t]) * C + c];
  }
}

__global__ void embedding_fwd_kernel(const float* __restrict__ w, const int64_t* __restrict__ ids, int B, int D,
                                     float* __restrict__ out) {
  const int b = blockIdx.x;
  for (int d = threadIdx.x; d < D; d += blockDim.x) out[(int64_t)b * D + d] = w[ids[b] * D + d];
}

// dense embedding gradient, deterministic: one thread per (row used, d), summing the batch in order
__global__ void embedding_bwd_kernel(const float* __restrict__ dout, const int64_t* __restrict__ ids, int B, int D,
                                     float* __restrict__ dw) {
  const int b = blockIdx.x;
  // only the first occurrence of each id accumulates all occurrences (in batch order)
  for (int p = 0; p < b; ++p)
    if (ids[p] == ids[b]) return;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f;
    for (int q = b; q < B; ++q)
      if (ids[q] == ids[b]) s += dout[(int64_t)q * D + d];
    dw[ids[b] * D + d] += s;
  }
}

// vqx_embedding_bwd_rows: block r = embedding row r; the batch's ids staged in
// LDS, every thread scans them in batch order and adds the matching rows of
// dout (one or two per id in a batch: a short load chain, not B serial loads)
constexpr int kEmbMaxB = 1024;
__global__ __launch_bounds__(256) void embedding_bwd_rows_kernel(const float* __restrict__ dout,
                                                                 const int64_t* __restrict__ ids, int B, int D,
                                                                 float* __restrict__ dw, int accumulate) {
  __shared__ int sid[kEmbMaxB];
  const int r = blockIdx.x;
  // batches above kEmbMaxB ids run in LDS-sized chunks (each chunk's sum added
  // to the row in chunk order; one chunk for B <= kEmbMaxB, as before)
  for (int q0 = 0; q0 < B; q0 += kEmbMaxB) {
    const int nq = min(kEmbMaxB, B - q0);
    __syncthreads();
    for (int q = threadIdx.x; q < nq; q += blockDim.x) sid[q] = (int)ids[q0 + q];
    __syncthreads();
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
      float s = 0.f;
      for (int q = 0; q < nq; ++q)
        if (sid[q] == r) s += dout[(int64_t)(q0 + q) * D + d];
      float* o = dw + (int64_t)r * D + d;
      *o = (accumulate || q0 > 0) ? *o + s : s;
    }
  }
}

__global__ void linear_fwd_kernel(const float* __restrict__ c, const float* __restrict__ W, const float* __restrict__ bias,
                                  int B, int I, int O, float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)B * O) return;
  const int b = (int)(e / O), o = (int)(e - (int64_t)b * O);
  float s = 0.f;
#pragma unroll 8
  for (int i = 0; i < I; ++i) s = fmaf(W[(int64_t)o * I + i], c[(int64_t)b * I + i], s);
  out[e] = s + (bias ? bias[o] : 0.f);
}

__global__ void linear_bwd_w_kernel(const float* __restrict__ dout, const float* __restrict__ c, int B, int I, int O,
                                    float* __restrict__ dW) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)O * I) return;
  const int o = (int)(e / I), i = (int)(e - (int64_t)o * I);
  float s = 0.f;
#pragma unroll 8
  for (int b = 0; b < B; ++b) s = fmaf(dout[(int64_t)b * O + o], c[(int64_t)b * I + i], s);
  dW[e] += s;
}

// dc[b][i] += sum_o dout[b][o] * W[o][i]: block (b, 64 columns i), 4 groups of o
__global__ __launch_bounds__(256) void linear_bwd_x_kernel(const float* __restrict__ dout, const float* __restrict__ W,
                                                           int B, int I, int O, float* __restrict__ dc) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int og = threadIdx.x >> 6;
  __shared__ float acc[4][64];
  float s = 0.f;
  if (i < I) {
    float s2 = 0.f;
    int o = og;
#pragma unroll 4
    for (; o + 4 < O; o += 8) {
      s = fmaf(dout[(int64_t)b * O + o], W[(int64_t)o * I + i], s);
      s2 = fmaf(dout[(int64_t)b * O + o + 4], W[(int64_t)(o + 4) * I + i], s2);
    }
    for (; o < O; o += 4) s = fmaf(dout[(int64_t)b * O + o], W[(int64_t)o * I + i], s);
    s += s2;
  }
  acc[og][threadIdx.x & 63] = s;
  __syncthreads();
  if (og == 0 && i < I) {
    const int l = threadIdx.x & 63;
    dc[(int64_t)b * I + i] += (acc[0][l] + acc[1][l]) + (acc[2][l] + acc[3][l]);
  }
}

// Batched speaker-conditioning linears (all ResSkip blocks per launch) as
// small LDS-tiled fp32 GEMMs: 64x64 output tiles, 256 threads x 16 outputs,
// K in chunks of 64.  Grid z carries (layer, tile of the third dimension).
constexpr int kLT = 64;

// out_l[b][o] = sum_i c[b][i] W_l[o][i] + bias_l[o].  grid (ceil(O/64), n, ceil(B/64))
__global__ __launch_bounds__(256) void linear_batched_fwd_kernel(const vqx_linear_layer* __restrict__ L,
                                                                 const float* __restrict__ c, int B, int I, int O) {
  const vqx_linear_layer& l = L[blockIdx.y];
  const int o0 = blockIdx.x * kLT, b0 = blockIdx.z * kLT;
  __shared__ float cs[kLT][kLT + 1];   // [b][i]
  __shared__ __attribute__((aligned(16))) float wt[kLT][kLT + 4];  // [i][o]
  const int t = threadIdx.x, tb = t >> 2, to = (t & 3) * 16;
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  for (int i0 = 0; i0 < I; i0 += kLT) {
    for (int e = t; e < kLT * kLT; e += 256) {
      const int r = e >> 6, q = e & 63;  // r: b or o row, q: i column (coalesced)
      cs[r][q] = (b0 + r < B && i0 + q < I) ? c[(int64_t)(b0 + r) * I + i0 + q] : 0.f;
      wt[q][r] = (o0 + r < O && i0 + q < I) ? l.W[(int64_t)(o0 + r) * I + i0 + q] : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int i = 0; i < kLT; ++i) {
      const float x = cs[tb][i];
#pragma unroll
      for (int j = 0; j < 16; j += 4) {
        const f32x4_t w = *(const f32x4_t*)&wt[i][to + j];
        acc[j] = fmaf(x, w[0], acc[j]);
        acc[j + 1] = fmaf(x, w[1], acc[j + 1]);
        acc[j + 2] = fmaf(x, w[2], acc[j + 2]);
        acc[j + 3] = fmaf(x, w[3], acc[j + 3]);
      }
    }
    __syncthreads();
  }
  const int b = b0 + tb;
  if (b >= B) return;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int o = o0 + to + j;
    if (o < O) l.out[(int64_t)b * O + o] = acc[j] + (l.bias ? l.bias[o] : 0.f);
  }
}

// dW_l[o][i] = sum_b dout_l[b][o] c[b][i]; dbias_l[o] = sum_b dout_l[b][o].
// grid (ceil(O/64), n, ceil(I/64)); the i-tile-0 blocks also write dbias.
__global__ __launch_bounds__(256) void linear_batched_bwd_w_kernel(const vqx_linear_layer* __restrict__ L,
                                                                   const float* __restrict__ c, int B, int I, int O) {
  const vqx_linear_layer& l = L[blockIdx.y];
  const int o0 = blockIdx.x * kLT, i0 = blockIdx.z * kLT;
  __shared__ float ds[kLT][kLT + 1];   // [b][o]
  __shared__ __attribute__((aligned(16))) float cs[kLT][kLT + 4];  // [b][i]
  const int t = threadIdx.x, to = t >> 2, ti = (t & 3) * 16;
  float acc[16], db = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  for (int b0 = 0; b0 < B; b0 += kLT) {
    for (int e = t; e < kLT * kLT; e += 256) {
      const int r = e >> 6, q = e & 63;
      ds[r][q] = (b0 + r < B && o0 + q < O) ? l.dout[(int64_t)(b0 + r) * O + o0 + q] : 0.f;
      cs[r][q] = (b0 + r < B && i0 + q < I) ? c[(int64_t)(b0 + r) * I + i0 + q] : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int b = 0; b < kLT; ++b) {
      const float d = ds[b][to];
      db += d;
#pragma unroll
      for (int j = 0; j < 16; j += 4) {
        const f32x4_t x = *(const f32x4_t*)&cs[b][ti + j];
        acc[j] = fmaf(d, x[0], acc[j]);
        acc[j + 1] = fmaf(d, x[1], acc[j + 1]);
        acc[j + 2] = fmaf(d, x[2], acc[j + 2]);
        acc[j + 3] = fmaf(d, x[3], acc[j + 3]);
      }
    }
    __syncthreads();
  }
  const int o = o0 + to;
  if (o >= O) return;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int i = i0 + ti + j;
    if (i < I) l.dW[(int64_t)o * I + i] = acc[j];
  }
  if (blockIdx.z == 0 && (t & 3) == 0 && l.dbias) l.dbias[o] = db;
}

// Split-K partial of dc[b][i] = sum_l sum_o dout_l[b][o] W_l[o][i] over one
// 64-wide o chunk of one layer.  grid (ceil(O/64), n, ceil(B/64)*ceil(I/64));
// part[(l*nO + oc)][b][i].
__global__ __launch_bounds__(256) void linear_batched_bwd_x_kernel(const vqx_linear_layer* __restrict__ L, int B,
                                                                   int I, int O, float* __restrict__ part) {
  const vqx_linear_layer& l = L[blockIdx.y];
  const float* __restrict__ dout = l.dout;
  const float* __restrict__ W = l.W;
  const int nI = (I + kLT - 1) / kLT;
  const int o0 = blockIdx.x * kLT, b0 = (blockIdx.z / nI) * kLT, i0 = (blockIdx.z % nI) * kLT;
  __shared__ float ds[kLT][kLT + 1];   // [b][o]
  __shared__ __attribute__((aligned(16))) float ws[kLT][kLT + 4];  // [o][i]
  const int t = threadIdx.x, tb = t >> 2, ti = (t & 3) * 16;
  // every operand load of the thread issued before the first is used (indices
  // clamped in range, the out-of-range elements zeroed at the LDS write): a
  // predicated load per element serialised them, one memory latency each
  constexpr int NE = kLT * kLT / 256;
  float dv[NE], wv[NE];
#pragma unroll
  for (int u = 0; u < NE; ++u) {
    const int e = t + 256 * u, r = e >> 6, q = e & 63;
    const int br = min(b0 + r, B - 1), oq = min(o0 + q, O - 1), orr = min(o0 + r, O - 1), iq = min(i0 + q, I - 1);
    dv[u] = dout[(int64_t)br * O + oq];
    wv[u] = W[(int64_t)orr * I + iq];
  }
#pragma unroll
  for (int u = 0; u < NE; ++u) {
    const int e = t + 256 * u, r = e >> 6, q = e & 63;
    ds[r][q] = (b0 + r < B && o0 + q < O) ? dv[u] : 0.f;
    ws[r][q] = (o0 + r < O && i0 + q < I) ? wv[u] : 0.f;
  }
  __syncthreads();
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
#pragma unroll 8
  for (int o = 0; o < kLT; ++o) {
    const float d = ds[tb][o];
#pragma unroll
    for (int j = 0; j < 16; j += 4) {
      const f32x4_t w = *(const f32x4_t*)&ws[o][ti + j];
      acc[j] = fmaf(d, w[0], acc[j]);
      acc[j + 1] = fmaf(d, w[1], acc[j + 1]);
      acc[j + 2] = fmaf(d, w[2], acc[j + 2]);
      acc[j + 3] = fmaf(d, w[3], acc[j + 3]);
    }
  }
  const int b = b0 + tb;
  if (b >= B) return;
  float* out = part + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * B * I;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int i = i0 + ti + j;
    if (i < I) out[(int64_t)b * I + i] = acc[j];
  }
}

// ---- speaker-conditioning fast path: I = 128 inputs, O % 64 == 0 (every
// recipe: cond dim 128); any B for the forward and the data gradient (their
// per-row results do not depend on B: data-parallel ranks and one process on
// the global batch agree row by row), B <= 64 for the weight gradient.  fp32 MFMA (v_mfma_f32_16x16x4f32, the
// reference's fp32): a workgroup is 4 waves x 16 output channels of one
// layer; the operands go straight from memory into the MFMA lane layout.  The
// K index is permuted so each lane's operands are contiguous: in step s, lane
// group q takes k = 32q + s (forward, K = I = 128) or b = 16q + s (weight
// gradient, K = B <= 64).  (Round 5: the LDS-blocked VALU kernels these
// replace took 11-12 us a launch, bound by three LDS reads per eight FMAs;
// the tiled kernels above, for other shapes, sum in a different order.)
constexpr int kCondI = 128, kCondB = 64, kCondO = 64;

// out_l[b][o] = bias_l[o] + sum_i c[b][i] W_l[o][i]; grid (O/64, n)
// ids != null: row b of c is row ids[b] of c (the embedding table: the lookup
// folded into the operand loads, vqx_linear_batched_fwd_ids)
__device__ __forceinline__ void linear_cond_fwd_block(const vqx_linear_layer* __restrict__ L,
                                                      const float* __restrict__ c, const int64_t* __restrict__ ids,
                                                      int B, int O, int bx, int layer) {
  const vqx_linear_layer& l = L[layer];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = lane >> 4, j = lane & 15;
  const int o0 = bx * kCondO + w * 16;
  // B operand (k = 32q + s, n = j): W[o0 + j][32q .. 32q + 31]
  f32x4_t wb[8];
  const float* wr = l.W + (int64_t)(o0 + j) * kCondI + 32 * q;
#pragma unroll
  for (int u = 0; u < 8; ++u) wb[u] = *(const f32x4_t*)(wr + 4 * u);
  const float bj = l.bias ? l.bias[o0 + j] : 0.f;
  for (int rt = 0; rt * 16 < B; ++rt) {
    // A operand (m = j, k = 32q + s): c[row][32q .. 32q + 31]; rows >= B read row B-1, not stored
    const int row = min(rt * 16 + j, B - 1);
    const float* cr = c + (ids ? ids[row] : (int64_t)row) * kCondI + 32 * q;
    f32x4_t ca[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) ca[u] = *(const f32x4_t*)(cr + 4 * u);
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ca[u][0], wb[u][0], acc, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(ca[u][1], wb[u][1], acc2, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ca[u][2], wb[u][2], acc, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(ca[u][3], wb[u][3], acc2, 0, 0, 0);
    }
    // D[m = 4q + r][n = j]
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = rt * 16 + 4 * q + r;
      if (b < B) l.out[(int64_t)b * O + o0 + j] = (acc[r] + acc2[r]) + bj;
    }
  }
}
__global__ __launch_bounds__(256) void linear_cond_fwd_kernel(const vqx_linear_layer* __restrict__ L,
                                                              const float* __restrict__ c,
                                                              const int64_t* __restrict__ ids, int B, int O) {
  linear_cond_fwd_block(L, c, ids, B, O, blockIdx.x, blockIdx.y);
}

// The training step's prologue in one launch (vqx_step_prologue): the
// conditioning linears (n_cond x O/64 blocks, latency-bound MFMA chains:
// first, so they start first), the input transpose (32 x 32 tiles), then the
// weight-norm pack units -- three independent jobs that ran as three
// launches in turn (11 + 5 + 22 us).  Each block runs the body of the
// launch it replaces, so the results are those launches' bits.
template <typename T>
__global__ __launch_bounds__(256) void step_prologue_kernel(const vqx_wn_layer* __restrict__ WL, WnUnits U,
                                                            const vqx_linear_layer* __restrict__ CL, int n_cond_blocks,
                                                            int cond_bx, const float* __restrict__ emb,
                                                            const int64_t* __restrict__ ids, int B, int O,
                                                            const float* __restrict__ x, int C, int T_, int tx_bx,
                                                            int tx_by, int n_tx_blocks, T* __restrict__ y, int ldy) {
  __shared__ __attribute__((aligned(16))) float buf[kWnBuf];
  __shared__ float red[16];
  int bid = (int)blockIdx.x;
  if (bid < n_cond_blocks) {
    linear_cond_fwd_block(CL, emb, ids, B, O, bid % cond_bx, bid / cond_bx);
    return;
  }
  bid -= n_cond_blocks;
  if (bid < n_tx_blocks) {
    const int r = bid / tx_bx;
    nct_to_ntc_tile<T>(x, C, T_, y, ldy, bid - r * tx_bx, r % tx_by, r / tx_by, (float(*)[33])buf);
    return;
  }
  wn_pack_block(WL, U, bid - n_tx_blocks, buf, red);
}

// dW_l[o][i] = sum_b dout_l[b][o] c[b][i], dbias_l[o] = sum_b dout_l[b][o]; grid (O/64, n)
// one workgroup (bx = output chunk, layer); cs: kCondB x kCondI floats of LDS (c, rows >= B zero)
__device__ __forceinline__ void linear_cond_bwd_w_block(const vqx_linear_layer* __restrict__ L,
                                                        const float* __restrict__ c, const int64_t* __restrict__ ids,
                                                        int B, int O, int bx, int layer, float (*cs)[kCondI]) {
  const vqx_linear_layer& l = L[layer];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = lane >> 4, j = lane & 15;
  const int o0 = bx * kCondO + w * 16;
  // A operand (m = j, k = b = 16q + s): dout[16q + s][o0 + j], zero past B
  float da[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int b = 16 * q + s;
    da[s] = l.dout[(int64_t)min(b, B - 1) * O + o0 + j];
  }
  constexpr int NC = kCondB * kCondI / 4 / 256;
  f32x4_t cv[NC];
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    const int e = threadIdx.x + 256 * u, r = e / (kCondI / 4), i4 = e % (kCondI / 4);
    const int row = min(r, B - 1);
    cv[u] = *(const f32x4_t*)(c + (ids ? ids[row] : (int64_t)row) * kCondI + 4 * i4);
  }
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    const int e = threadIdx.x + 256 * u, r = e / (kCondI / 4), i4 = e % (kCondI / 4);
    const f32x4_t z = {0.f, 0.f, 0.f, 0.f};
    *(f32x4_t*)&cs[r][4 * i4] = r < B ? cv[u] : z;
  }
  // dbias: the lane's 16 rows in order, then the four lane groups (q) in order
  float db = 0.f;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    if (16 * q + s >= B) da[s] = 0.f;
    db += da[s];
  }
  {
    const float d1 = __shfl(db, j + 16, 64), d2 = __shfl(db, j + 32, 64), d3 = __shfl(db, j + 48, 64);
    if (q == 0 && l.dbias) l.dbias[o0 + j] = ((db + d1) + d2) + d3;
  }
  __syncthreads();
  for (int it = 0; it < kCondI / 16; ++it) {
    // B operand (k = b = 16q + s, n = j): c[16q + s][16 it + j]
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 16; s += 2) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(da[s], cs[16 * q + s][16 * it + j], acc, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(da[s + 1], cs[16 * q + s + 1][16 * it + j], acc2, 0, 0, 0);
    }
    // D[m = 4q + r][n = j]: dW[o0 + 4q + r][16 it + j]
#pragma unroll
    for (int r = 0; r < 4; ++r) l.dW[(int64_t)(o0 + 4 * q + r) * kCondI + 16 * it + j] = acc[r] + acc2[r];
  }
}
__global__ __launch_bounds__(256) void linear_cond_bwd_w_kernel(const vqx_linear_layer* __restrict__ L,
                                                                const float* __restrict__ c,
                                                                const int64_t* __restrict__ ids, int B, int O) {
  __shared__ float cs[kCondB][kCondI];
  linear_cond_bwd_w_block(L, c, ids, B, O, blockIdx.x, blockIdx.y, cs);
}

// dc partials: part[l * (O/64) + oc][b][i] = sum over the chunk's 64 outputs o
// of dout_l[b][o] W_l[o][i] (k = o = o0 + 16q + s); sum_slices_wide_kernel adds
// the slices in order.  Wave w covers inputs 32w .. 32w + 31.  grid (O/64, n)
__device__ __forceinline__ void linear_cond_bwd_x_block(const vqx_linear_layer* __restrict__ L, int B, int O,
                                                        float* __restrict__ part, int bx, int layer) {
  const vqx_linear_layer& l = L[layer];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = lane >> 4, j = lane & 15;
  const int o0 = bx * kCondO;
  const int64_t slice = (int64_t)layer * (O / kCondO) + bx;
  // B operand (k = 16q + s, n = j) of the wave's two 16-input tiles
  float wv[2][16];
#pragma unroll
  for (int it = 0; it < 2; ++it)
#pragma unroll
    for (int s = 0; s < 16; ++s) wv[it][s] = l.W[(int64_t)(o0 + 16 * q + s) * kCondI + 32 * w + 16 * it + j];
  for (int rt = 0; rt * 16 < B; ++rt) {
    // A operand (m = j, k = 16q + s): dout[row][o0 + 16q + s]; rows >= B read row B-1, not stored
    const float* dr = l.dout + (int64_t)min(rt * 16 + j, B - 1) * O + o0 + 16 * q;
    float da[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) da[s] = dr[s];
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 16; s += 2) {
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(da[s], wv[it][s], acc, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(da[s + 1], wv[it][s + 1], acc2, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = rt * 16 + 4 * q + r;
        if (b < B) part[(slice * B + b) * kCondI + 32 * w + 16 * it + j] = acc[r] + acc2[r];
      }
    }
  }
}
__global__ __launch_bounds__(256) void linear_cond_bwd_x_kernel(const vqx_linear_layer* __restrict__ L, int B, int O,
                                                                float* __restrict__ part) {
  linear_cond_bwd_x_block(L, B, O, part, blockIdx.x, blockIdx.y);
}
// both in one grid (O/64, 2n): layers' dW / dbias in y < n, their dc slices in y >= n
__global__ __launch_bounds__(256) void linear_cond_bwd_kernel(const vqx_linear_layer* __restrict__ L,
                                                              const float* __restrict__ c,
                                                              const int64_t* __restrict__ ids, int B, int O, int n,
                                                              float* __restrict__ part) {
  __shared__ float cs[kCondB][kCondI];
  if ((int)blockIdx.y < n) linear_cond_bwd_w_block(L, c, ids, B, O, blockIdx.x, blockIdx.y, cs);
  else linear_cond_bwd_x_block(L, B, O, part, blockIdx.x, blockIdx.y - n);
}

// dc[e] = sum_p part[p][e] in a fixed order: each of the 4 waves of a
// workgroup sums a contiguous quarter of the slices (8 loads in flight) for
// 64 elements, then the quarters are added in order (deterministic).
__global__ __launch_bounds__(256) void sum_slices_wide_kernel(const float* __restrict__ part, int np, int64_t n,
                                                              float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int q = threadIdx.x >> 6;
  const int p0 = (int)((int64_t)np * q / 4), p1 = (int)((int64_t)np * (q + 1) / 4);
  __shared__ float red[4][64];
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (e < n) {
    int p = p0;
    for (; p + 8 <= p1; p += 8) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = part[(int64_t)(p + u) * n + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += t[u];
    }
    for (int u = 0; p < p1; ++p, ++u) a[u] += part[(int64_t)p * n + e];
  }
  red[q][threadIdx.x & 63] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (q == 0 && e < n) out[e] = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// dc[e] = sum_p part[p][e] in a fixed order (deterministic)
__global__ __launch_bounds__(256) void sum_slices_kernel(const float* __restrict__ part, int np, int64_t n,
                                                         float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int p = 0;
  for (; p + 4 <= np; p += 4) {
    a0 += part[(int64_t)p * n + e];
    a1 += part[(int64_t)(p + 1) * n + e];
    a2 += part[(int64_t)(p + 2) * n + e];
    a3 += part[(int64_t)(p + 3) * n + e];
  }
  for (; p < np; ++p) a0 += part[(int64_t)p * n + e];
  out[e] = (a0 + a1) + (a2 + a3);
}

// --------------------------------------------------------------- optimizer
constexpr int kNormBlocks = 1024;

__global__ __launch_bounds__(256) void sqnorm_partial_kernel(const float* __restrict__ g, int64_t n,
                                                             float* __restrict__ part) {
  __shared__ float red[16];
  float s = 0.f;
  const int64_t n4 = n / 4;
  const f32x4_t* g4 = (const f32x4_t*)g;
#pragma unroll 4
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const f32x4_t v = g4[i];
    s = fmaf(v[0], v[0], s); s = fmaf(v[1], v[1], s); s = fmaf(v[2], v[2], s); s = fmaf(v[3], v[3], s);
  }
  if (blockIdx.x == 0)
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) s = fmaf(g[i], g[i], s);
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// The global gradient norm from the weight-norm backward's partials
// (vqx_weight_norm_bwd_sq) and g^2 over the ranges [off, off+len) it did not
// write: kSqBlocks blocks each sum a fixed strided share of both into
// scratch[b], then one block adds the kSqBlocks values in order into out[0].
// Deterministic (fixed assignment and order).
constexpr int kSqBlocks = 256;  // one per CU: 64 left the pass at 9.6 us, latency-bound
__global__ __launch_bounds__(256) void sq_partial_sum_kernel(const float* __restrict__ part, int64_t np,
                                                             const float* __restrict__ g,
                                                             const int64_t* __restrict__ rng, int nr,
                                                             float* __restrict__ scratch) {
  __shared__ float red[16];
  const int64_t stride = (int64_t)kSqBlocks * 256;
  const int64_t j0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  // the first ranges' bounds load beside the partials (one latency, not one per range)
  constexpr int kR = 8;
  int64_t ro[kR], rl[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const int rr = min(r, max(nr - 1, 0));
    ro[r] = nr ? rng[2 * rr] : 0;
    rl[r] = r < nr ? rng[2 * rr + 1] : 0;
  }
  float s = 0.f;
  // partials four at a time, clamped loads (no tail loop of single loads), added in index order
  for (int64_t i = j0; i < np; i += 4 * stride) {
    float t[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) t[u] = part[min(i + u * stride, np - 1)];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * stride < np) s += t[u];
  }
  // each range's first element of this thread loaded together, then the ranges in order
  float gv[kR];
  if (nr > 0) {  // (g may be null without ranges)
#pragma unroll
    for (int r = 0; r < kR; ++r) gv[r] = g[ro[r] + min(j0, max(rl[r] - 1, (int64_t)0))];
  }
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    if (r >= nr) break;
    if (j0 < rl[r]) s = fmaf(gv[r], gv[r], s);
    for (int64_t j = j0 + stride; j < rl[r]; j += stride) s = fmaf(g[ro[r] + j], g[ro[r] + j], s);
  }
  for (int r = kR; r < nr; ++r) {
    const int64_t off = rng[2 * r], len = rng[2 * r + 1];
    for (int64_t j = j0; j < len; j += stride) s = fmaf(g[off + j], g[off + j], s);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) scratch[blockIdx.x] = s;
}
// Adam's per-step scalars (StepLR'd lr, bias corrections) from the device step
// counter, which it advances; one thread
__device__ __forceinline__ void adam_hyper_eval(int64_t* __restrict__ step, double lr0, double gamma, int step_size,
                                                double b1, double b2, double eps, float* __restrict__ hyper) {
  const int64_t t = step[0] + 1;
  step[0] = t;
  const double lr = lr0 * pow(gamma, (double)((t - 1) / step_size));
  const double bc1 = 1.0 - pow(b1, (double)t);
  const double bc2 = 1.0 - pow(b2, (double)t);
  hyper[0] = (float)lr;
  hyper[1] = (float)(lr / bc1);
  hyper[2] = (float)sqrt(bc2);
  hyper[3] = (float)t;
  hyper[4] = (float)(1.0 - b1);
  hyper[5] = (float)b2;
  hyper[6] = (float)(1.0 - b2);
  hyper[7] = (float)eps;
}

__global__ void adam_hyper_kernel(int64_t* __restrict__ step, double lr0, double gamma, int step_size, double b1,
                                  double b2, double eps, float* __restrict__ hyper) {
  adam_hyper_eval(step, lr0, gamma, step_size, b1, b2, eps, hyper);
}

// the second level of vqx_sq_norm_finish; with hyper != null (vqx_sq_norm_finish_adam)
// thread 0 also evaluates Adam's per-step scalars: one launch fewer
struct AdamHyperArgs {
  int64_t* step;
  double lr0, gamma, b1, b2, eps;
  int step_size;
  float* hyper;
};
__global__ __launch_bounds__(kSqBlocks) void sq_final_kernel(const float* __restrict__ scratch, float* __restrict__ out,
                                                             AdamHyperArgs H) {
  __shared__ float red[16];
  const float s = block_sum(scratch[threadIdx.x], red);
  if (threadIdx.x == 0) {
    out[0] = s;
    if (H.hyper) adam_hyper_eval(H.step, H.lr0, H.gamma, H.step_size, H.b1, H.b2, H.eps, H.hyper);
  }
}

// RAdam (trainer/radam.py:15-78): rectification decided once per step on the
// device, in double like the reference's Python floats.
__global__ void radam_hyper_kernel(int64_t* __restrict__ step, double lr0, double gamma, int step_size, double b1,
                                   double b2, double eps, float* __restrict__ hyper) {
  const int64_t t = step[0] + 1;
  step[0] = t;
  const double lr = lr0 * pow(gamma, (double)((t - 1) / step_size));
  const double b2t = pow(b2, (double)t);
  const double nmax = 2.0 / (1.0 - b2) - 1.0;
  const double nsma = nmax - 2.0 * (double)t * b2t / (1.0 - b2t);
  const bool rect = nsma >= 5.0;
  const double ss = rect ? sqrt((1.0 - b2t) * (nsma - 4.0) / (nmax - 4.0) * (nsma - 2.0) / nsma * nmax / (nmax - 2.0)) /
                               (1.0 - pow(b1, (double)t))
                         : 1.0 / (1.0 - pow(b1, (double)t));
  hyper[0] = (float)lr;
  hyper[1] = (float)(-ss * lr);
  hyper[2] = rect ? 1.f : 0.f;
  hyper[3] = (float)t;
  hyper[4] = (float)b1;
  hyper[5] = (float)(1.0 - b1);
  hyper[6] = (float)b2;
  hyper[7] = (float)(1.0 - b2);
  hyper[8] = (float)eps;
}

__global__ __launch_bounds__(256) void radam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                    const float* __restrict__ hyper, const float* __restrict__ sumsq,
                                                    float max_norm) {
  float coef = 1.f;
  if (max_norm > 0.f && sumsq) {
    const float tn = sqrtf(sumsq[0]);
    coef = max_norm / (tn + 1e-6f);
    coef = coef < 1.f ? coef : 1.f;
  }
  const float val = hyper[1];
  const bool rect = hyper[2] != 0.f;
  const float b1 = hyper[4], omb1 = hyper[5], b2 = hyper[6], omb2 = hyper[7], eps = hyper[8];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = __fmul_rn(g[i], coef);
    float vi = __fmul_rn(v[i], b2);
    vi = __fadd_rn(vi, __fmul_rn(__fmul_rn(omb2, gi), gi));      // addcmul_(g, g, value=1-b2)
    float mi = __fadd_rn(__fmul_rn(m[i], b1), __fmul_rn(omb1, gi));  // mul_(b1).add_(g, alpha=1-b1)
    const float upd = rect ? __fdiv_rn(mi, __fadd_rn(__fsqrt_rn(vi), eps)) : mi;
    p[i] = __fadd_rn(p[i], __fmul_rn(val, upd));
    m[i] = mi;
    v[i] = vi;
  }
}

// One Adam element update in torch's op order (torch.optim.Adam single-tensor,
// trainer/basic.py:63-75).  Plain operators under contract(off): every product
// and sum is rounded on its own, so the 16-B path and the scalar path agree bit
// for bit.  The pragma holds because the library is built with
// -ffp-contract=fast-honor-pragmas (plain "fast" lets the backend fuse across
// it: the packed path then carried v_pk_fma_f32 and differed by an ulp).
// Against torch's CPU Adam the bound is 1e-6 relative (its vectorised
// lerp/addcmul may fuse).
__device__ __forceinline__ void adam_elem(float& pi, float gi, float& mi, float& vi, float w, float b2, float omb2,
                                          float bc2s, float eps, float step_size) {
#pragma clang fp contract(off)
  // torch.lerp: weight < 0.5 ? m + w*(g-m) : g - (g-m)*(1-w)
  mi = (w < 0.5f) ? mi + w * (gi - mi) : gi - (gi - mi) * (1.f - w);
  vi = vi * b2;
  vi = vi + (omb2 * gi) * gi;
  const float den = __fsqrt_rn(vi) / bc2s + eps;
  pi = pi + (-step_size) * (mi / den);
}

// 16-B accesses (4 elements per thread per step, 16 loads in flight) when all
// four buffers are 16-B aligned, else one element at a time; the tail is scalar.
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                   const float* __restrict__ hyper, const float* __restrict__ sumsq,
                                                   float max_norm) {
  float coef = 1.f;
  if (max_norm > 0.f && sumsq) {
    const float tn = sqrtf(sumsq[0]);
    coef = max_norm / (tn + 1e-6f);
    coef = coef < 1.f ? coef : 1.f;
  }
  const float step_size = hyper[1], bc2s = hyper[2];
  const float w = hyper[4], b2 = hyper[5], omb2 = hyper[6], eps = hyper[7];
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (int64_t)gridDim.x * blockDim.x;
  int64_t done = 0;
  if ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0) {
    const int64_t n4 = n >> 2;
    for (int64_t i = tid; i < n4; i += nth) {
      f32x4_t pv = ((const f32x4_t*)p)[i], gv = ((const f32x4_t*)g)[i];
      f32x4_t mv = ((const f32x4_t*)m)[i], vv = ((const f32x4_t*)v)[i];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pi = pv[e], mi = mv[e], vi = vv[e];
        adam_elem(pi, __fmul_rn(gv[e], coef), mi, vi, w, b2, omb2, bc2s, eps, step_size);
        pv[e] = pi;
        mv[e] = mi;
        vv[e] = vi;
      }
      ((f32x4_t*)p)[i] = pv;
      ((f32x4_t*)m)[i] = mv;
      ((f32x4_t*)v)[i] = vv;
    }
    done = n4 << 2;
  }
  for (int64_t i = done + tid; i < n; i += nth) {
    float pi = p[i], mi = m[i], vi = v[i];
    adam_elem(pi, __fmul_rn(g[i], coef), mi, vi, w, b2, omb2, bc2s, eps, step_size);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

// Adam with the next forward's weight-norm preparation fused in
// (vqx_adam_step_wn).  Blocks [0, row_off[n_layers]) own the rows of the
// weight-normed convs in the table: each updates its rows of v = weight_v
// and their gains weight_g[o] (adam_elem, the bits of adam_kernel), reduces
// ||v_o|| of the NEW row in the canonical order of the pack (kind 0, k > 1:
// 256-thread block, thread t the elements 4t + 1024u + (0..3); kind 0 k = 1
// and kind 1: a wave per row, lane l the elements 4l + 256u + (0..3); nested
// fmaf of the four, then block / wave sums), stores it in norm[o] and, for
// kind 0 (Conv1d), writes the packed w = g*v/||v|| exactly as wn_pack_kernel
// would from the same parameters.  The remaining blocks update the flat
// segments (start, len) of everything else, 4096 elements a block.
constexpr int kAdamMaxL = 128, kAdamMaxS = 128;
struct AdamWnPlan {
  int n_layers, n_segs;
  int row_off[kAdamMaxL + 1];  // block prefix of the row layers
  int seg_blk[kAdamMaxS + 1];  // block prefix of the flat segments (after the row blocks)
};
__host__ __device__ inline int adam_wn_units(const vqx_wn_layer& l) {
  return l.kind == 1 ? l.cin : l.k > 1 ? l.cout : (l.cout + 3) / 4;
}
struct AdamHyper {
  float coef, step_size, bc2s, w, b2, omb2, eps;
};
__device__ __forceinline__ AdamHyper adam_hyper_load(const float* hyper, const float* sumsq, float max_norm) {
  AdamHyper h;
  h.coef = 1.f;
  if (max_norm > 0.f && sumsq) {
    const float tn = sqrtf(sumsq[0]);
    h.coef = max_norm / (tn + 1e-6f);
    h.coef = h.coef < 1.f ? h.coef : 1.f;
  }
  h.step_size = hyper[1];
  h.bc2s = hyper[2];
  h.w = hyper[4];
  h.b2 = hyper[5];
  h.omb2 = hyper[6];
  h.eps = hyper[7];
  return h;
}
__device__ __forceinline__ f32x4_t adam4(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                         float* __restrict__ v, int64_t i, const AdamHyper& h) {
  f32x4_t pv = *(const f32x4_t*)(p + i), gv = *(const f32x4_t*)(g + i);
  f32x4_t mv = *(const f32x4_t*)(m + i), vv = *(const f32x4_t*)(v + i);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float pi = pv[e], mi = mv[e], vi = vv[e];
    adam_elem(pi, __fmul_rn(gv[e], h.coef), mi, vi, h.w, h.b2, h.omb2, h.bc2s, h.eps, h.step_size);
    pv[e] = pi;
    mv[e] = mi;
    vv[e] = vi;
  }
  *(f32x4_t*)(p + i) = pv;
  *(f32x4_t*)(m + i) = mv;
  *(f32x4_t*)(v + i) = vv;
  return pv;
}
__device__ __forceinline__ float adam1(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                       float* __restrict__ v, int64_t i, const AdamHyper& h) {
  float pi = p[i], mi = m[i], vi = v[i];
  adam_elem(pi, __fmul_rn(g[i], h.coef), mi, vi, h.w, h.b2, h.omb2, h.bc2s, h.eps, h.step_size);
  p[i] = pi;
  m[i] = mi;
  v[i] = vi;
  return pi;
}
__device__ __forceinline__ float sq4(const f32x4_t x, float s) {
  return fmaf(x[0], x[0], fmaf(x[1], x[1], fmaf(x[2], x[2], fmaf(x[3], x[3], s))));
}

__global__ __launch_bounds__(256, 4) void adam_wn_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v,
                                                      const float* __restrict__ hyper,
                                                      const float* __restrict__ sumsq, float max_norm,
                                                      const vqx_wn_layer* __restrict__ L,
                                                      const int64_t* __restrict__ segs, AdamWnPlan P) {
  const AdamHyper h = adam_hyper_load(hyper, sumsq, max_norm);
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (b >= P.row_off[P.n_layers]) {  // flat segment chunk: 4096 elements
    int lo = 0, hi = P.n_segs - 1;
    const int rb = b - P.row_off[P.n_layers];
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (P.seg_blk[mid] <= rb) lo = mid; else hi = mid - 1;
    }
    const int64_t s0 = segs[2 * lo], len = segs[2 * lo + 1];
    const int64_t c0 = (int64_t)(rb - P.seg_blk[lo]) * 4096;
    if ((s0 & 3) == 0 && (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t j = c0 + (int64_t)threadIdx.x * 4 + 1024 * u;
        if (j + 4 <= len) {
          adam4(p, g, m, v, s0 + j, h);
        } else {
          for (int64_t e = j; e < len && e < j + 4; ++e) adam1(p, g, m, v, s0 + e, h);
        }
      }
    } else {
      for (int64_t j = c0 + threadIdx.x; j < len && j < c0 + 4096; j += 256) adam1(p, g, m, v, s0 + j, h);
    }
    return;
  }
  int lo = 0, hi = P.n_layers - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (P.row_off[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const vqx_wn_layer& l = L[lo];
  const int unit = b - P.row_off[lo];
  const int K = l.k, cin = l.cin, cout = l.cout;
  const int64_t voff = l.v - p, goff = l.g - p;
  if (l.kind == 1 || K > 1) {
    // one row per 256-thread block: Conv1d row co (packed [co][j*cin + ci]
    // through LDS) or ConvT row ci (norm only); every load of the thread's
    // elements is issued before the first update
    __shared__ __attribute__((aligned(16))) float buf[kWnRow];
    __shared__ float red[16];
    __shared__ float gnew;
    const int o = unit;
    const int cols = l.kind == 1 ? cout * K : cin * K;
    const int64_t r0 = voff + (int64_t)o * cols;
    constexpr int U = kWnRow / 1024, UC = 2;  // UC 16-B groups' loads in flight at a time (register budget)
    float s = 0.f;
#pragma unroll
    for (int u0 = 0; u0 < U; u0 += UC) {
      f32x4_t pv[UC], gv[UC], mv[UC], vv[UC];
#pragma unroll
      for (int uu = 0; uu < UC; ++uu) {
        const int i = (int)threadIdx.x * 4 + 1024 * (u0 + uu);
        if (i < cols) {
          pv[uu] = *(const f32x4_t*)(p + r0 + i);
          gv[uu] = *(const f32x4_t*)(g + r0 + i);
          mv[uu] = *(const f32x4_t*)(m + r0 + i);
          vv[uu] = *(const f32x4_t*)(v + r0 + i);
        }
      }
#pragma unroll
      for (int uu = 0; uu < UC; ++uu) {
        const int i = (int)threadIdx.x * 4 + 1024 * (u0 + uu);
        if (i < cols) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float pi = pv[uu][e], mi = mv[uu][e], vi = vv[uu][e];
            adam_elem(pi, __fmul_rn(gv[uu][e], h.coef), mi, vi, h.w, h.b2, h.omb2, h.bc2s, h.eps, h.step_size);
            pv[uu][e] = pi;
            mv[uu][e] = mi;
            vv[uu][e] = vi;
          }
          *(f32x4_t*)(p + r0 + i) = pv[uu];
          *(f32x4_t*)(m + r0 + i) = mv[uu];
          *(f32x4_t*)(v + r0 + i) = vv[uu];
          if (l.kind == 0) *(f32x4_t*)(buf + i) = pv[uu];
          s = sq4(pv[uu], s);
        }
      }
    }
    if (threadIdx.x == 0) gnew = adam1(p, g, m, v, goff + o, h);
    s = block_sum(s, red);  // its barriers publish buf and gnew
    const float nrm = sqrtf(s);
    if (threadIdx.x == 0) l.norm[o] = nrm;
    if (l.kind == 1) return;
    const int co = o;
    const float sc = gnew / nrm;
    bf16_t* wb = (bf16_t*)l.w_packed + (int64_t)co * cols;
    if (l.dtype == VQX_BF16 && (cin & 3) == 0 && (((uintptr_t)wb) & 7) == 0) {
      for (int e = threadIdx.x * 4; e < cols; e += 1024) {  // 4 consecutive ci of one tap, 8 B a lane
        const int j = e / cin, ci = e - j * cin;
        const float* bb = buf + ci * K + j;
        *(uint2*)(wb + e) = make_uint2(pack_bf16x2(bb[0] * sc, bb[K] * sc), pack_bf16x2(bb[2 * K] * sc, bb[3 * K] * sc));
      }
      return;
    }
    for (int e = threadIdx.x; e < cols; e += 256) {
      const int j = e / cin, ci = e - j * cin;
      st_dt(l.w_packed, (int64_t)co * cols + e, buf[ci * K + j] * sc, l.dtype);
    }
    return;
  }
  // a wave per row: kind 0 k = 1 (row co of cin, packed = the row scaled)
  const int o = unit * 4 + wv;
  if (o >= cout) return;
  const int cols = cin;
  const int64_t r0 = voff + (int64_t)o * cols;
  float s = 0.f;
  {
    f32x4_t xs[2], gv[2], mv[2], vv[2];  // cols <= 512
#pragma unroll
    for (int u = 0; u < 2; ++u) {  // every load first
      const int i = lane * 4 + 256 * u;
      if (i < cols) {
        xs[u] = *(const f32x4_t*)(p + r0 + i);
        gv[u] = *(const f32x4_t*)(g + r0 + i);
        mv[u] = *(const f32x4_t*)(m + r0 + i);
        vv[u] = *(const f32x4_t*)(v + r0 + i);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = lane * 4 + 256 * u;
      if (i < cols) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float pi = xs[u][e], mi = mv[u][e], vi = vv[u][e];
          adam_elem(pi, __fmul_rn(gv[u][e], h.coef), mi, vi, h.w, h.b2, h.omb2, h.bc2s, h.eps, h.step_size);
          xs[u][e] = pi;
          mv[u][e] = mi;
          vv[u][e] = vi;
        }
        *(f32x4_t*)(p + r0 + i) = xs[u];
        *(f32x4_t*)(m + r0 + i) = mv[u];
        *(f32x4_t*)(v + r0 + i) = vv[u];
        s = sq4(xs[u], s);
      }
    }
    float gn = 0.f;
    if (lane == 0) gn = adam1(p, g, m, v, goff + o, h);
    gn = __shfl(gn, 0, 64);
    s = wave_sum(s);
    const float nrm = sqrtf(s);
    if (lane == 0) l.norm[o] = nrm;
    const float sc = gn / nrm;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = lane * 4 + 256 * u;
      if (i < cols) {
        const f32x4_t x = xs[u];
        if (l.dtype == VQX_BF16) {
          *(uint2*)((bf16_t*)l.w_packed + (int64_t)o * cols + i) =
              make_uint2(pack_bf16x2(x[0] * sc, x[1] * sc), pack_bf16x2(x[2] * sc, x[3] * sc));
        } else {
          *(f32x4_t*)((float*)l.w_packed + (int64_t)o * cols + i) = f32x4_t{x[0] * sc, x[1] * sc, x[2] * sc, x[3] * sc};
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void scale_act_2d_kernel(const void* __restrict__ src, int lds, int sdt,
                                                           void* __restrict__ dst, int ldd, int ddt, int64_t rows,
                                                           int cols, float scale, int act) {
  const int64_t total = rows * cols;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / cols;
    const int c = (int)(e - r * cols);
    float v = scale * ld_dt(src, r * lds + c, sdt);
    if (act == VQX_PRO_RELU) v = v > 0.f ? v : 0.f;
    else if (act == VQX_PRO_LRELU) v = v > 0.f ? v : 0.2f * v;
    st_dt(dst, r * ldd + c, v, ddt);
  }
}

__global__ __launch_bounds__(256) void convert_2d_kernel(const void* __restrict__ src, int lds, int sdt,
                                                         void* __restrict__ dst, int ldd, int ddt, int64_t rows,
                                                         int cols) {
  const int64_t total = rows * cols;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / cols;
    const int c = (int)(e - r * cols);
    const float v = src ? ld_dt(src, r * lds + c, sdt) : 0.f;
    st_dt(dst, r * ldd + c, v, ddt);
  }
}

// convert_2d / scale_act_2d on 8-element chunks (cols, both leading
// dimensions multiples of 8, 16-B aligned rows): 16-B bf16 / 2 x 16-B f32
// accesses, four chunks' loads in flight per thread, 32-bit chunk indexing
// (the element kernels above divide 64-bit indices and move 2-4 B a lane).
template <typename S> struct Chunk8;
template <> struct Chunk8<float> {
  __device__ static __forceinline__ void ld(const float* p, float* f) {
    const f32x4_t a = *(const f32x4_t*)p, b = *(const f32x4_t*)(p + 4);
    f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3]; f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
  }
  __device__ static __forceinline__ void st(float* p, const float* f) {
    *(f32x4_t*)p = f32x4_t{f[0], f[1], f[2], f[3]};
    *(f32x4_t*)(p + 4) = f32x4_t{f[4], f[5], f[6], f[7]};
  }
};
template <> struct Chunk8<bf16_t> {
  __device__ static __forceinline__ void ld(const bf16_t* p, float* f) { Vec<bf16_t>::load(p, f); }
  __device__ static __forceinline__ void st(bf16_t* p, const float* f) { Vec<bf16_t>::store(p, f); }
};
// zdst (optional): a second matrix (n8z chunks, cprz per row) set to zero in the
// same launch (vqx_convert_2d_zero2): chunk indices past n8 address it
template <typename S, typename D, bool ZERO>
__global__ __launch_bounds__(256) void map8_kernel(const S* __restrict__ src, int lds, D* __restrict__ dst, int ldd,
                                                   int n8, int cpr, float scale, int act, D* __restrict__ zdst,
                                                   int ldz, int n8z, int cprz) {
  constexpr int U = 4;
  const int stride = gridDim.x * 256;
  const int total = n8 + n8z;
  for (int q0 = blockIdx.x * 256 + threadIdx.x; q0 < total; q0 += U * stride) {
    float v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = q0 + u * stride;
      if (ZERO || q >= n8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[u][k] = 0.f;
      } else {
        const int r = q / cpr, c = (q - r * cpr) * 8;
        Chunk8<S>::ld(src + (int64_t)r * lds + c, v[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = q0 + u * stride;
      if (q >= total) break;
      if (q < n8) {
        const int r = q / cpr, c = (q - r * cpr) * 8;
        if (!ZERO) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            float x = scale * v[u][k];
            if (act == VQX_PRO_RELU) x = x > 0.f ? x : 0.f;
            else if (act == VQX_PRO_LRELU) x = x > 0.f ? x : 0.2f * x;
            v[u][k] = x;
          }
        }
        Chunk8<D>::st(dst + (int64_t)r * ldd + c, v[u]);
      } else {
        const int qz = q - n8, r = qz / cprz, c = (qz - r * cprz) * 8;
        Chunk8<D>::st(zdst + (int64_t)r * ldz + c, v[u]);  // zeros
      }
    }
  }
}

}  // namespace vqx

using namespace vqx;

static int grid_for(int64_t n, int block = 256, int cap = 8192) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

// the pack kernel's limits on a host table; returns the most ConvT rows (the
// norm pre-pass's grid) or -1 with the error set
static int wn_fwd_check(const vqx_wn_layer* lh, int32_t n_layers, const char* who) {
  int max_t_rows = 1;
  for (int i = 0; i < n_layers; ++i) {
    const vqx_wn_layer& l = lh[i];
    if (l.kind != 0 && l.kind != 1 && l.kind != VQX_WN_RESAMPLE && l.kind != VQX_WN_RESAMPLE_T) { set_error("%s: layer %d bad kind", who, i); return -1; }
    if (l.kind >= VQX_WN_RESAMPLE && !(l.stride >= 1 && l.pad >= 0 && l.pad <= l.stride && l.k - 1 - l.pad < 2 * l.stride)) { set_error("%s: layer %d: resampling conv needs 0 <= pad <= stride and k-1-pad < 2*stride", who, i); return -1; }
    const bool rsm = l.kind >= VQX_WN_RESAMPLE;
    const bool row_is_cout = l.kind == 0 || l.kind == VQX_WN_RESAMPLE;
    if ((row_is_cout ? l.cin : l.cout) * l.k > kWnRow || (!rsm && l.k > 64)) { set_error("%s: layer %d row too long", who, i); return -1; }
    if (l.kind == 1) max_t_rows = l.cin > max_t_rows ? l.cin : max_t_rows;
  }
  return max_t_rows;
}

static int wn_fwd_launch(const vqx_wn_layer* lh, const vqx_wn_layer* ld, int32_t n_layers, int32_t flags,
                         vqx_stream_t stream) {
  if (!lh || !ld || n_layers <= 0) { set_error("vqx_weight_norm_fwd: bad tables"); return -1; }
  const int max_t_rows = wn_fwd_check(lh, n_layers, "vqx_weight_norm_fwd");
  if (max_t_rows < 0) return -1;
  hipStream_t s = (hipStream_t)stream;
  if (!(flags & VQX_WNF_NORMS_READY))
    hipLaunchKernelGGL(wn_norm_kernel, dim3(max_t_rows, n_layers), dim3(256), 0, s, ld, n_layers);
  for (int i0 = 0; i0 < n_layers; i0 += kWnMaxL) {  // flat grid over the layers' units, kWnMaxL layers a launch
    WnUnits U;
    U.n = n_layers - i0 < kWnMaxL ? n_layers - i0 : kWnMaxL;
    U.off[0] = 0;
    for (int i = 0; i < U.n; ++i) U.off[i + 1] = U.off[i] + wn_pack_units(lh[i0 + i]);
    if (U.off[U.n] > 0) hipLaunchKernelGGL(wn_pack_kernel, dim3(U.off[U.n]), dim3(256), 0, s, ld + i0, U);
  }
  return launch_status("vqx_weight_norm_fwd");
}

extern "C" int vqx_weight_norm_fwd(const vqx_wn_layer* lh, const vqx_wn_layer* ld, int32_t n_layers,
                                   vqx_stream_t stream) {
  return wn_fwd_launch(lh, ld, n_layers, 0, stream);
}

extern "C" int vqx_weight_norm_fwd_flags(const vqx_wn_layer* lh, const vqx_wn_layer* ld, int32_t n_layers,
                                         int32_t flags, vqx_stream_t stream) {
  return wn_fwd_launch(lh, ld, n_layers, flags, stream);
}

static int wn_bwd_units(const vqx_wn_layer& l) {
  return l.kind == VQX_WN_COLREDUCE ? (l.cout + kWnCrCols - 1) / kWnCrCols
         : wn_bwd_wave_rows(l)       ? (l.cout + kWnThreads / 64 - 1) / (kWnThreads / 64)
         : (l.kind == 0 || l.kind == VQX_WN_RESAMPLE) ? l.cout
                                                      : l.cin;
}

extern "C" int vqx_weight_norm_bwd_partials(const vqx_wn_layer* lh, int32_t n_layers, int64_t* count) {
  if (!lh || n_layers <= 0 || !count) { set_error("vqx_weight_norm_bwd_partials: bad arguments"); return -1; }
  int64_t b = 0;
  for (int i = 0; i < n_layers; ++i) b += wn_bwd_units(lh[i]);
  *count = b * (kWnThreads / 64);
  return 0;
}

static int wn_bwd_launch(const vqx_wn_layer* lh, const vqx_wn_layer* ld, int32_t n_layers, float* sq,
                         int64_t sq_capacity, vqx_stream_t stream) {
  if (!lh || !ld || n_layers <= 0) { set_error("vqx_weight_norm_bwd: bad tables"); return -1; }
  if (sq) {
    int64_t need = 0;
    vqx_weight_norm_bwd_partials(lh, n_layers, &need);
    if (sq_capacity < need) { set_error("vqx_weight_norm_bwd_sq: %lld partials < %lld", (long long)sq_capacity, (long long)need); return -1; }
  }
  int max_rows = 1;
  for (int i = 0; i < n_layers; ++i) {
    const vqx_wn_layer& l = lh[i];
    if (l.kind == VQX_WN_COLREDUCE) {
      if (!l.v || !l.dv || l.cin < 1 || l.cout < 1) { set_error("vqx_weight_norm_bwd: column-reduce entry %d", i); return -1; }
      const int blocks = (l.cout + 255) / 256;
      max_rows = blocks > max_rows ? blocks : max_rows;
      continue;
    }
    if (l.kind != 0 && l.kind != 1 && l.kind != VQX_WN_RESAMPLE && l.kind != VQX_WN_RESAMPLE_T) { set_error("vqx_weight_norm_bwd: layer %d bad kind", i); return -1; }
    if (l.kind >= VQX_WN_RESAMPLE && !(l.stride >= 1 && l.pad >= 0 && l.pad <= l.stride && l.k - 1 - l.pad < 2 * l.stride)) { set_error("vqx_weight_norm_bwd: layer %d: bad resampling geometry", i); return -1; }
    const bool row_is_cout = l.kind == 0 || l.kind == VQX_WN_RESAMPLE;
    const int rows = row_is_cout ? l.cout : l.cin;
    const int cols = (row_is_cout ? l.cin : l.cout) * l.k;
    if (cols > 4096) { set_error("vqx_weight_norm_bwd: row length %d > 4096", cols); return -1; }
    if (!l.slabs || !l.dv || (l.g && !l.dg) || l.splits < 1) { set_error("vqx_weight_norm_bwd: layer %d missing buffers", i); return -1; }
    if ((row_is_cout ? l.cin : l.cout) % 4 || ((uintptr_t)l.slabs & 15)) { set_error("vqx_weight_norm_bwd: layer %d: slab rows must be 16-B vectors", i); return -1; }
    if (l.slab_dtype != VQX_F32 && l.slab_dtype != VQX_BF16) { set_error("vqx_weight_norm_bwd: layer %d: slab_dtype %d", i, l.slab_dtype); return -1; }
    max_rows = rows > max_rows ? rows : max_rows;
  }
  (void)max_rows;
  for (int i0 = 0; i0 < n_layers; i0 += kWnMaxL) {  // flat grid over the layers' rows, kWnMaxL layers a launch
    WnUnits U;
    U.n = n_layers - i0 < kWnMaxL ? n_layers - i0 : kWnMaxL;
    U.off[0] = 0;
    for (int i = 0; i < U.n; ++i) U.off[i + 1] = U.off[i] + wn_bwd_units(lh[i0 + i]);
    if (U.off[U.n] > 0)
      hipLaunchKernelGGL(wn_bwd_kernel, dim3(U.off[U.n]), dim3(kWnThreads), 0, (hipStream_t)stream, ld + i0, U, sq);
    if (sq) sq += (int64_t)U.off[U.n] * (kWnThreads / 64);
  }
  return launch_status("vqx_weight_norm_bwd");
}

extern "C" int vqx_weight_norm_bwd(const vqx_wn_layer* lh, const vqx_wn_layer* ld, int32_t n_layers,
                                   vqx_stream_t stream) {
  return wn_bwd_launch(lh, ld, n_layers, nullptr, 0, stream);
}

extern "C" int vqx_weight_norm_bwd_sq(const vqx_wn_layer* lh, const vqx_wn_layer* ld, int32_t n_layers,
                                      float* sq_partials, int64_t sq_capacity, vqx_stream_t stream) {
  if (!sq_partials) { set_error("vqx_weight_norm_bwd_sq: null partials"); return -1; }
  return wn_bwd_launch(lh, ld, n_layers, sq_partials, sq_capacity, stream);
}

extern "C" int vqx_sq_norm_finish(const float* partials, int64_t n_partials, const float* g, const int64_t* ranges,
                                  int32_t n_ranges, float* scratch, float* out, vqx_stream_t stream) {
  if (n_partials < 0 || n_ranges < 0 || !out || !scratch || (n_partials && !partials) || (n_ranges && (!ranges || !g))) {
    set_error("vqx_sq_norm_finish: bad arguments");
    return -1;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sq_partial_sum_kernel, dim3(kSqBlocks), dim3(256), 0, s, partials, n_partials, g, ranges, n_ranges,
                     scratch);
  hipLaunchKernelGGL(sq_final_kernel, dim3(1), dim3(kSqBlocks), 0, s, scratch, out, AdamHyperArgs{});
  return launch_status("vqx_sq_norm_finish");
}

extern "C" int vqx_sq_norm_finish_adam(const float* partials, int64_t n_partials, const float* g,
                                       const int64_t* ranges, int32_t n_ranges, float* scratch, float* out,
                                       int64_t* step, double lr0, double gamma, int32_t step_size, double beta1,
                                       double beta2, double eps, float* hyper, vqx_stream_t stream) {
  if (n_partials < 0 || n_ranges < 0 || !out || !scratch || (n_partials && !partials) || (n_ranges && (!ranges || !g)) ||
      !step || !hyper || step_size < 1) {
    set_error("vqx_sq_norm_finish_adam: bad arguments");
    return -1;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sq_partial_sum_kernel, dim3(kSqBlocks), dim3(256), 0, s, partials, n_partials, g, ranges, n_ranges,
                     scratch);
  hipLaunchKernelGGL(sq_final_kernel, dim3(1), dim3(kSqBlocks), 0, s, scratch, out,
                     AdamHyperArgs{step, lr0, gamma, beta1, beta2, eps, step_size, hyper});
  return launch_status("vqx_sq_norm_finish_adam");
}

extern "C" int vqx_groupnorm_stats(const void* x, int32_t ldx, int32_t dtype, int64_t n_rows, int32_t T, int32_t C,
                                   int32_t G, float eps, float* partials, float* mean_rstd, vqx_stream_t stream) {
  if (G < 1 || C % G || n_rows % T) { set_error("vqx_groupnorm_stats: bad shape"); return -1; }
  const int B = (int)(n_rows / T);
  hipStream_t s = (hipStream_t)stream;
  const int V = dtype == VQX_BF16 ? 8 : 4;
  const int cg = C / G, cpr = cg / V;
  const bool vec = (cg % V == 0) && (ldx % V == 0) && cpr <= 256 && (256 % cpr == 0) && (((uintptr_t)x & 15) == 0);
  if (dtype == VQX_BF16) {
    if (vec) hipLaunchKernelGGL(gn_partial_vec_kernel<bf16_t>, dim3(kGnParts, B * G), dim3(256), 0, s, (const bf16_t*)x, ldx, T, C, G, cpr, partials);
    else hipLaunchKernelGGL(gn_partial_kernel<bf16_t>, dim3(kGnParts, B * G), dim3(256), 0, s, (const bf16_t*)x, ldx, T, C, G, partials);
  } else {
    if (vec) hipLaunchKernelGGL(gn_partial_vec_kernel<float>, dim3(kGnParts, B * G), dim3(256), 0, s, (const float*)x, ldx, T, C, G, cpr, partials);
    else hipLaunchKernelGGL(gn_partial_kernel<float>, dim3(kGnParts, B * G), dim3(256), 0, s, (const float*)x, ldx, T, C, G, partials);
  }
  hipLaunchKernelGGL(gn_finalize_kernel, dim3((B * G + 127) / 128), dim3(128), 0, s, partials, B * G, eps, mean_rstd);
  return launch_status("vqx_groupnorm_stats");
}

static int gn_glu_fwd_impl(const void* u, int32_t ldu, void* g, int32_t ldg, int32_t dtype, int64_t n_rows,
                           int32_t T, int32_t C, const float* mean_rstd, const float* gamma, const float* beta,
                           const float* tiles, float eps, float* mr_out, vqx_stream_t stream);

extern "C" int vqx_gn_glu_fwd(const void* u, int32_t ldu, void* g, int32_t ldg, int32_t dtype, int64_t n_rows,
                              int32_t T, int32_t C, const float* mean_rstd, const float* gamma, const float* beta,
                              vqx_stream_t stream) {
  return gn_glu_fwd_impl(u, ldu, g, ldg, dtype, n_rows, T, C, mean_rstd, gamma, beta, nullptr, 0.f, nullptr, stream);
}

extern "C" int vqx_gn_glu_fwd_tiles(const void* u, int32_t ldu, void* g, int32_t ldg, int32_t dtype, int64_t n_rows,
                                    int32_t T, int32_t C, const float* parts, float eps, float* mean_rstd,
                                    const float* gamma, const float* beta, vqx_stream_t stream) {
  if (!parts || !mean_rstd || T % 128 || n_rows % T || C % 256) {
    set_error("vqx_gn_glu_fwd_tiles: needs T %% 128 == 0 and C %% 256 == 0");
    return -1;
  }
  return gn_glu_fwd_impl(u, ldu, g, ldg, dtype, n_rows, T, C, nullptr, gamma, beta, parts, eps, mean_rstd, stream);
}

static int gn_glu_fwd_impl(const void* u, int32_t ldu, void* g, int32_t ldg, int32_t dtype, int64_t n_rows,
                           int32_t T, int32_t C, const float* mean_rstd, const float* gamma, const float* beta,
                           const float* tiles, float eps, float* mr_out, vqx_stream_t stream) {
  if (C % 2) { set_error("vqx_gn_glu_fwd: odd C"); return -1; }
  const int V = dtype == VQX_BF16 ? 8 : 4;
  if ((C / 2) % V || ldu % V || ldg % V || (((uintptr_t)u | (uintptr_t)g) & 15)) {
    set_error("vqx_gn_glu_fwd: channels/strides must be multiples of %d", V);
    return -1;
  }
  const int cpr = (C / 2) / V;
  if (cpr > 256 || 256 % cpr) { set_error("vqx_gn_glu_fwd: C/2/%d must divide 256", V); return -1; }
  // frames per workgroup: every workgroup of the in-launch-statistics path
  // merges its utterance's GEMM tiles first, so larger blocks amortise that
  const int fpb = 16;  // frames per workgroup (4/8/32/64 measured slower: profiles/r02/glu_fpb_ab.txt)
  const int grid = (int)((n_rows + fpb - 1) / fpb);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == VQX_BF16)
    hipLaunchKernelGGL(gn_glu_fwd_vec_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)u, ldu, (bf16_t*)g, ldg, (int)n_rows, T, C / 2, cpr, mean_rstd, gamma, beta, tiles, eps, mr_out, fpb);
  else
    hipLaunchKernelGGL(gn_glu_fwd_vec_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)u, ldu, (float*)g, ldg, (int)n_rows, T, C / 2, cpr, mean_rstd, gamma, beta, tiles, eps, mr_out, fpb);
  return launch_status("vqx_gn_glu_fwd");
}

extern "C" int vqx_gn_lrelu_fwd(const void* h, int32_t ldh, void* g, int32_t ldg, int32_t dtype, int64_t n_rows,
                                int32_t T, int32_t C, const float* mean_rstd, const float* gamma, const float* beta,
                                vqx_stream_t stream) {
  const int V = dtype == VQX_BF16 ? 8 : 4;
  if (!h || !g || !mean_rstd || !gamma || !beta || T < 1 || n_rows % T || C % V || ldh % V || ldg % V ||
      (((uintptr_t)h | (uintptr_t)g) & 15)) {
    set_error("vqx_gn_lrelu_fwd: bad arguments (C, strides multiples of %d, 16-B aligned)", V);
    return -1;
  }
  const int cpr = C / V;
  const int64_t total = n_rows * cpr;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 4096);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == VQX_BF16)
    hipLaunchKernelGGL(gn_lrelu_fwd_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)h, ldh, (bf16_t*)g, ldg,
                       n_rows, T, cpr, mean_rstd, gamma, beta);
  else
    hipLaunchKernelGGL(gn_lrelu_fwd_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)h, ldh, (float*)g, ldg,
                       n_rows, T, cpr, mean_rstd, gamma, beta);
  return launch_status("vqx_gn_lrelu_fwd");
}

extern "C" int vqx_gn_bwd(const void* dy, int32_t lddy, const void* u, int32_t ldu, void* du, int32_t lddu,
                          int32_t dtype, int64_t n_rows, int32_t T, int32_t C, int32_t G, int32_t glu,
                          const float* mean_rstd, const float* gamma, const float* beta, float* partials,
                          int32_t nparts, float* colsum_p, float* dgamma_p, float* dbeta_p, vqx_stream_t stream) {
  if (nparts < 0) { set_error("vqx_gn_bwd: nparts < 0"); return -1; }
  if (glu && G != 2) { set_error("vqx_gn_bwd: glu requires G=2"); return -1; }
  if (!glu && G != 1) { set_error("vqx_gn_bwd: non-glu path supports G=1"); return -1; }
  if (C % G || n_rows % T) { set_error("vqx_gn_bwd: bad shape"); return -1; }
  const int B = (int)(n_rows / T);
  const int V = dtype == VQX_BF16 ? 8 : 4;
  const int span = glu ? C / 2 : C;  // channels covered by the chunk index
  const int cpr = span / V;
  if (span % V || lddy % V || ldu % V || lddu % V || cpr > 256 || 256 % cpr ||
      (((uintptr_t)dy | (uintptr_t)u | (uintptr_t)du) & 15)) {
    set_error("vqx_gn_bwd: channel count / strides must give a power-of-two chunk count <= 256 (C=%d)", C);
    return -1;
  }
  hipStream_t s = (hipStream_t)stream;
  // nparts == 0: reduce here (kGnBwdParts row parts per utterance, G*2 floats
  // each); nparts > 0: the producing GEMM's GNBWD epilogue already wrote
  // nparts tiles per utterance (4 floats each)
  const int np = nparts ? nparts : kGnBwdParts, ps = nparts ? 4 : G * 2;
  if (dtype == VQX_BF16) {
    if (!nparts) hipLaunchKernelGGL(gn_bwd_reduce_vec_kernel<bf16_t>, dim3(kGnBwdParts, B), dim3(256), 0, s, (const bf16_t*)dy, lddy, (const bf16_t*)u, ldu, T, C, G, glu, cpr, mean_rstd, gamma, beta, partials);
    auto* kfn = glu ? gn_bwd_apply_vec_kernel<bf16_t, true> : gn_bwd_apply_vec_kernel<bf16_t, false>;
    hipLaunchKernelGGL(kfn, dim3((cpr * 2 + 15) / 16, B), dim3(512), 0, s, (const bf16_t*)dy, lddy, (const bf16_t*)u, ldu, (bf16_t*)du, lddu, T, C, G, glu, cpr, mean_rstd, gamma, beta, partials, np, ps, colsum_p, dgamma_p, dbeta_p);
  } else {
    if (!nparts) hipLaunchKernelGGL(gn_bwd_reduce_vec_kernel<float>, dim3(kGnBwdParts, B), dim3(256), 0, s, (const float*)dy, lddy, (const float*)u, ldu, T, C, G, glu, cpr, mean_rstd, gamma, beta, partials);
    auto* kfn = glu ? gn_bwd_apply_vec_kernel<float, true> : gn_bwd_apply_vec_kernel<float, false>;
    hipLaunchKernelGGL(kfn, dim3((cpr + 15) / 16, B), dim3(512), 0, s, (const float*)dy, lddy, (const float*)u, ldu, (float*)du, lddu, T, C, G, glu, cpr, mean_rstd, gamma, beta, partials, np, ps, colsum_p, dgamma_p, dbeta_p);
  }
  return launch_status("vqx_gn_bwd");
}

// row parts of the first colsum level and the vector kernel's lanes per row group
static int colsum_geometry(int64_t n_rows, int C, int dtype, int* lanes) {
  const int V = dtype == VQX_BF16 ? 8 : 4;
  int L = 1;  // lanes per row group in the vector kernel: pow2 >= C/V, <= 32
  while (L < 32 && L * V < C) L <<= 1;
  const int colblocks = (C + V * L - 1) / (V * L);  // >= 1 for any C > 0
  int nparts = (256 + colblocks - 1) / colblocks;
  if (nparts > 64) nparts = 64;
  if (nparts > n_rows / 8) nparts = (int)(n_rows / 8);
  if (nparts < 1) nparts = 1;
  if (lanes) *lanes = L;
  return nparts;
}

// first level: partials[p][c] over nparts row parts
static void colsum_partials_launch(const void* x, int ldx, int dtype, int64_t n_rows, int C, int nparts, int L,
                                   float* partials, hipStream_t s) {
  const int V = dtype == VQX_BF16 ? 8 : 4;
  const bool vec = (C % V == 0) && (ldx % V == 0) && (((uintptr_t)x & 15) == 0);
  if (vec) {
    const int nch = C / V;
    if (dtype == VQX_BF16)
      hipLaunchKernelGGL(colsum_partial_vec_kernel<bf16_t>, dim3((nch + L - 1) / L, nparts), dim3(256), 0, s, (const bf16_t*)x, ldx, n_rows, C, nparts, L, partials);
    else
      hipLaunchKernelGGL(colsum_partial_vec_kernel<float>, dim3((nch + L - 1) / L, nparts), dim3(256), 0, s, (const float*)x, ldx, n_rows, C, nparts, L, partials);
  } else if (dtype == VQX_BF16) {
    hipLaunchKernelGGL(colsum_partial_kernel<bf16_t>, dim3((C + 63) / 64, nparts), dim3(256), 0, s, (const bf16_t*)x, ldx, n_rows, C, nparts, partials);
  } else {
    hipLaunchKernelGGL(colsum_partial_kernel<float>, dim3((C + 63) / 64, nparts), dim3(256), 0, s, (const float*)x, ldx, n_rows, C, nparts, partials);
  }
}

extern "C" int vqx_colsum_parts(int64_t n_rows, int32_t C, int32_t dtype, int32_t* nparts) {
  if (n_rows <= 0 || C <= 0 || !nparts) { set_error("vqx_colsum_parts: bad arguments"); return -1; }
  *nparts = colsum_geometry(n_rows, C, dtype, nullptr);
  return 0;
}

extern "C" int vqx_colsum_partials(const void* x, int32_t ldx, int32_t dtype, int64_t n_rows, int32_t C,
                                   float* partials, vqx_stream_t stream) {
  if (!x || !partials || n_rows <= 0 || C <= 0 || ldx < C) { set_error("vqx_colsum_partials: bad arguments"); return -1; }
  int L = 1;
  const int nparts = colsum_geometry(n_rows, C, dtype, &L);
  colsum_partials_launch(x, ldx, dtype, n_rows, C, nparts, L, partials, (hipStream_t)stream);
  return launch_status("vqx_colsum_partials");
}

extern "C" int vqx_colsum(const void* x, int32_t ldx, int32_t dtype, int64_t n_rows, int32_t C, float* partials,
                          float* out, int32_t accumulate, vqx_stream_t stream) {
  if (n_rows <= 0 || C <= 0) { set_error("vqx_colsum: bad shape"); return -1; }
  hipStream_t s = (hipStream_t)stream;
  if (n_rows <= 64) {
    if (dtype == VQX_BF16)
      hipLaunchKernelGGL(colsum_small_kernel<bf16_t>, dim3((C + 63) / 64), dim3(256), 0, s, (const bf16_t*)x, ldx, n_rows, C, out, accumulate);
    else
      hipLaunchKernelGGL(colsum_small_kernel<float>, dim3((C + 63) / 64), dim3(256), 0, s, (const float*)x, ldx, n_rows, C, out, accumulate);
    return launch_status("vqx_colsum");
  }
  int L = 1;
  const int nparts = colsum_geometry(n_rows, C, dtype, &L);
  colsum_partials_launch(x, ldx, dtype, n_rows, C, nparts, L, partials, s);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((C + 3) / 4), dim3(256), 0, s, partials, nparts, C, out, accumulate);
  return launch_status("vqx_colsum");
}

extern "C" int vqx_nct_to_ntc(const float* x, int32_t B, int32_t C, int32_t T, void* y, int32_t ldy, int32_t dtype,
                              vqx_stream_t stream) {
  dim3 grid((T + 31) / 32, (C + 31) / 32, B);
  if (dtype == VQX_BF16)
    hipLaunchKernelGGL(nct_to_ntc_kernel<bf16_t>, grid, dim3(256), 0, (hipStream_t)stream, x, B, C, T, (bf16_t*)y, ldy);
  else
    hipLaunchKernelGGL(nct_to_ntc_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, x, B, C, T, (float*)y, ldy);
  return launch_status("vqx_nct_to_ntc");
}

extern "C" int vqx_ntc_to_nct(const void* y, int32_t ldy, int32_t dtype, int32_t B, int32_t C, int32_t T, float* x,
                              vqx_stream_t stream) {
  dim3 grid((T + 31) / 32, (C + 31) / 32, B);
  if (dtype == VQX_BF16)
    hipLaunchKernelGGL(ntc_to_nct_kernel<bf16_t>, grid, dim3(256), 0, (hipStream_t)stream, (const bf16_t*)y, ldy, B, C, T, x);
  else
    hipLaunchKernelGGL(ntc_to_nct_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, (const float*)y, ldy, B, C, T, x);
  return launch_status("vqx_ntc_to_nct");
}

// loss_out == NULL: the partials only (their count in *n_parts), summed by the caller's later launch
static int logloss_impl(const float* x, const float* xhat, int32_t ldxh, int32_t B, int32_t C, int32_t T,
                        float grad_scale, void* dxhat, int32_t lddx, int32_t dtype, float* loss_out, float* partials,
                        const float* extra_parts, int32_t n_extra, float* extra_out, vqx_stream_t stream,
                        int32_t* n_parts = nullptr) {
  const int64_t total = (int64_t)B * C * T;
  if (total <= 0 || total >= (1LL << 31)) { set_error("vqx_logloss_fwd_bwd: B*C*T must be in [1, 2^31)"); return -1; }
  hipStream_t s = (hipStream_t)stream;
  const int tiles = (T + kLlTile - 1) / kLlTile;
  const uintptr_t dx_align = dtype == VQX_BF16 ? 7 : 15;  // 4-element chunks: 8-B bf16 / 16-B f32 stores
  int grid;
  if (C % 4 == 0 && ldxh % 4 == 0 && (!dxhat || lddx % 4 == 0) && C <= 256 && (int64_t)tiles * B <= 1024 &&
      ((uintptr_t)xhat & 15) == 0 && (!dxhat || ((uintptr_t)dxhat & dx_align) == 0)) {
    grid = tiles * B;  // partials: at most 1024 (the caller's buffer)
    const size_t lds = (size_t)C * (kLlTile + 1) * sizeof(float);
    if (dtype == VQX_BF16)
      hipLaunchKernelGGL(logloss_tile_kernel<bf16_t>, dim3(tiles, B), dim3(256), lds, s, x, xhat, ldxh, C, T, grad_scale, (bf16_t*)dxhat, lddx, partials);
    else
      hipLaunchKernelGGL(logloss_tile_kernel<float>, dim3(tiles, B), dim3(256), lds, s, x, xhat, ldxh, C, T, grad_scale, (float*)dxhat, lddx, partials);
  } else {
    grid = grid_for(total, 256, 1024);
    if (dtype == VQX_BF16)
      hipLaunchKernelGGL(logloss_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, x, xhat, ldxh, B, C, T, grad_scale, (bf16_t*)dxhat, lddx, partials);
    else
      hipLaunchKernelGGL(logloss_kernel<float>, dim3(grid), dim3(256), 0, s, x, xhat, ldxh, B, C, T, grad_scale, (float*)dxhat, lddx, partials);
  }
  if (n_parts) *n_parts = grid;
  if (!loss_out) return launch_status("vqx_logloss_parts");
  if (extra_parts)
    hipLaunchKernelGGL(sum_partials2_kernel, dim3(1), dim3(1024), 0, s, partials, grid, 1.0f / ((float)B * (float)T),
                       loss_out, extra_parts, n_extra, 1.0f, extra_out);
  else
    hipLaunchKernelGGL(sum_partials_scale_kernel, dim3(1), dim3(1024), 0, s, partials, grid, 1.0f / ((float)B * (float)T), loss_out);
  return launch_status("vqx_logloss_fwd_bwd");
}

extern "C" int vqx_logloss_fwd_bwd(const float* x, const float* xhat, int32_t ldxh, int32_t B, int32_t C, int32_t T,
                                   float grad_scale, void* dxhat, int32_t lddx, int32_t dtype, float* loss_out,
                                   float* partials, vqx_stream_t stream) {
  return logloss_impl(x, xhat, ldxh, B, C, T, grad_scale, dxhat, lddx, dtype, loss_out, partials, nullptr, 0, nullptr,
                      stream);
}

extern "C" int vqx_logloss_parts(const float* x, const float* xhat, int32_t ldxh, int32_t B, int32_t C, int32_t T,
                                 float grad_scale, void* dxhat, int32_t lddx, int32_t dtype, float* partials,
                                 int32_t* n_parts, vqx_stream_t stream) {
  if (!partials || !n_parts) { set_error("vqx_logloss_parts: needs partials and n_parts"); return -1; }
  return logloss_impl(x, xhat, ldxh, B, C, T, grad_scale, dxhat, lddx, dtype, nullptr, partials, nullptr, 0, nullptr,
                      stream, n_parts);
}

extern "C" int vqx_logloss_fwd_bwd_x(const float* x, const float* xhat, int32_t ldxh, int32_t B, int32_t C, int32_t T,
                                     float grad_scale, void* dxhat, int32_t lddx, int32_t dtype, float* loss_out,
                                     float* partials, const float* extra_partials, int32_t n_extra, float* extra_out,
                                     vqx_stream_t stream) {
  if (!extra_partials || !extra_out || n_extra < 1) {
    set_error("vqx_logloss_fwd_bwd_x: needs extra partials and their output");
    return -1;
  }
  return logloss_impl(x, xhat, ldxh, B, C, T, grad_scale, dxhat, lddx, dtype, loss_out, partials, extra_partials,
                      n_extra, extra_out, stream);
}

extern "C" int vqx_time_gather(const void* x, void* y, int32_t B, int32_t T, int32_t C, const int32_t* src_t,
                               int32_t dtype, vqx_stream_t stream) {
  if ((int64_t)B * T * C >= (1LL << 31)) { set_error("vqx_time_gather: B*T*C must be < 2^31"); return -1; }
  const int grid = grid_for((int64_t)B * T * C);
  if (dtype == VQX_BF16)
    hipLaunchKernelGGL(time_gather_kernel<bf16_t>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, (bf16_t*)y, B, T, C, src_t);
  else
    hipLaunchKernelGGL(time_gather_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float*)x, (float*)y, B, T, C, src_t);
  return launch_status("vqx_time_gather");
}

extern "C" int vqx_embedding_fwd(const float* weight, const int64_t* ids, int32_t B, int32_t D, float* out,
                                 vqx_stream_t stream) {
  hipLaunchKernelGGL(embedding_fwd_kernel, dim3(B), dim3(128), 0, (hipStream_t)stream, weight, ids, B, D, out);
  return launch_status("vqx_embedding_fwd");
}

extern "C" int vqx_embedding_bwd(const float* dout, const int64_t* ids, int32_t B, int32_t D, float* dweight,
                                 vqx_stream_t stream) {
  hipLaunchKernelGGL(embedding_bwd_kernel, dim3(B), dim3(128), 0, (hipStream_t)stream, dout, ids, B, D, dweight);
  return launch_status("vqx_embedding_bwd");
}

extern "C" int vqx_embedding_bwd_rows(const float* dout, const int64_t* ids, int32_t B, int32_t D, int32_t n_rows,
                                      float* dweight, int32_t accumulate, vqx_stream_t stream) {
  if (!dout || !ids || !dweight || B < 1 || D < 1 || n_rows < 1) {
    set_error("vqx_embedding_bwd_rows: bad arguments");
    return -1;
  }
  hipLaunchKernelGGL(embedding_bwd_rows_kernel, dim3(n_rows), dim3(D >= 256 ? 256 : ((D + 63) / 64) * 64), 0,
                     (hipStream_t)stream, dout, ids, B, D, dweight, accumulate);
  return launch_status("vqx_embedding_bwd_rows");
}

extern "C" int vqx_linear_f32(const float* c, const float* W, const float* bias, int32_t B, int32_t I, int32_t O,
                              float* out, vqx_stream_t stream) {
  hipLaunchKernelGGL(linear_fwd_kernel, dim3(grid_for((int64_t)B * O, 256, 1 << 20)), dim3(256), 0, (hipStream_t)stream, c, W, bias, B, I, O, out);
  return launch_status("vqx_linear_f32");
}

extern "C" int vqx_linear_bwd_f32(const float* dout, const float* c, const float* W, int32_t B, int32_t I, int32_t O,
                                  float* dW, float* dc, vqx_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dW) hipLaunchKernelGGL(linear_bwd_w_kernel, dim3(grid_for((int64_t)O * I, 256, 1 << 20)), dim3(256), 0, s, dout, c, B, I, O, dW);
  if (dc) hipLaunchKernelGGL(linear_bwd_x_kernel, dim3((I + 63) / 64, B), dim3(256), 0, s, dout, W, B, I, O, dc);
  return launch_status("vqx_linear_bwd_f32");
}

extern "C" int vqx_grad_sq_norm(const float* g, int64_t n, float* partials, float* out, vqx_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sqnorm_partial_kernel, dim3(kNormBlocks), dim3(256), 0, s, g, n, partials);
  hipLaunchKernelGGL(sum_partials_scale_kernel, dim3(1), dim3(1024), 0, s, partials, kNormBlocks, 1.0f, out);
  return launch_status("vqx_grad_sq_norm");
}

extern "C" int vqx_adam_hyper(int64_t* step, double lr0, double gamma, int32_t step_size, double beta1,
                              double beta2, double eps, float* hyper, vqx_stream_t stream) {
  if (step_size < 1) { set_error("vqx_adam_hyper: step_size < 1"); return -1; }
  hipLaunchKernelGGL(adam_hyper_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, step, lr0, gamma, step_size, beta1,
                     beta2, eps, hyper);
  return launch_status("vqx_adam_hyper");
}

extern "C" int vqx_adam_step(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper,
                             const float* sumsq, float max_norm, vqx_stream_t stream) {
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for((n + 3) / 4, 256, 4096)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n,
                     hyper, sumsq, max_norm);
  return launch_status("vqx_adam_step");
}

extern "C" int vqx_adam_step_wn(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper,
                                const float* sumsq, float max_norm, const vqx_wn_layer* rows_host,
                                const vqx_wn_layer* rows_dev, int32_t n_layers, const int64_t* segs_host,
                                const int64_t* segs_dev, int32_t n_segs, vqx_stream_t stream) {
  if (!p || !g || !m || !v || !hyper || n_layers < 0 || n_segs < 0 || n_layers > kAdamMaxL || n_segs > kAdamMaxS ||
      (n_layers && (!rows_host || !rows_dev)) || (n_segs && (!segs_host || !segs_dev))) {
    set_error("vqx_adam_step_wn: bad arguments (at most %d layers and %d segments)", kAdamMaxL, kAdamMaxS);
    return -1;
  }
  // the row path moves 16-B vectors of p, g, m, v (the segment path checks its own alignment)
  if ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) {
    set_error("vqx_adam_step_wn: p, g, m and v must be 16-B aligned");
    return -1;
  }
  AdamWnPlan P;
  P.n_layers = n_layers;
  P.n_segs = n_segs;
  P.row_off[0] = 0;
  int64_t covered = 0;
  // every interval the launch updates (v and g rows of each layer, the flat
  // segments), to check that they do not overlap (with the coverage count
  // below: exactly once each of the n elements)
  int64_t iv[2 * (2 * kAdamMaxL + kAdamMaxS)];
  int niv = 0;
  for (int i = 0; i < n_layers; ++i) {
    const vqx_wn_layer& l = rows_host[i];
    const bool k3 = l.kind == 0 && l.k > 1;
    const int cols = l.kind == 0 ? l.cin * l.k : l.cout * l.k;
    const int rows = l.kind == 0 ? l.cout : l.cin;
    const int64_t vo = l.v - p, go = l.g - p;
    const bool ok = (l.kind == 0 || l.kind == 1) && l.g && l.norm && (l.kind == 1 || l.w_packed) && l.k >= 1 &&
                    cols % 4 == 0 && cols <= (k3 || l.kind == 1 ? kWnRow : 512) && vo >= 0 && vo % 4 == 0 &&
                    vo + (int64_t)rows * cols <= n && go >= 0 && go + rows <= n &&
                    (l.dtype == VQX_BF16 || l.dtype == VQX_F32) &&
                    (l.kind == 1 || k3 ||
                     ((((uintptr_t)l.w_packed) & 15) == 0 && (l.cin * (l.dtype == VQX_BF16 ? 2 : 4)) % 16 == 0));
    if (!ok) { set_error("vqx_adam_step_wn: layer %d cannot take the fused weight-norm preparation", i); return -1; }
    P.row_off[i + 1] = P.row_off[i] + adam_wn_units(l);
    covered += (int64_t)rows * cols + rows;
    iv[2 * niv] = vo; iv[2 * niv + 1] = vo + (int64_t)rows * cols; ++niv;
    iv[2 * niv] = go; iv[2 * niv + 1] = go + rows; ++niv;
  }
  P.seg_blk[0] = 0;
  for (int i = 0; i < n_segs; ++i) {
    const int64_t s0 = segs_host[2 * i], len = segs_host[2 * i + 1];
    if (s0 < 0 || len < 0 || s0 + len > n) { set_error("vqx_adam_step_wn: segment %d out of range", i); return -1; }
    P.seg_blk[i + 1] = P.seg_blk[i] + (int)((len + 4095) / 4096);
    covered += len;
    if (len > 0) { iv[2 * niv] = s0; iv[2 * niv + 1] = s0 + len; ++niv; }
  }
  // insertion sort by start (at most 2 * 128 + 128 intervals), then adjacent overlap test
  for (int i = 1; i < niv; ++i)
    for (int j = i; j > 0 && iv[2 * j] < iv[2 * (j - 1)]; --j) {
      const int64_t a0 = iv[2 * j], a1 = iv[2 * j + 1];
      iv[2 * j] = iv[2 * (j - 1)]; iv[2 * j + 1] = iv[2 * (j - 1) + 1];
      iv[2 * (j - 1)] = a0; iv[2 * (j - 1) + 1] = a1;
    }
  for (int i = 1; i < niv; ++i)
    if (iv[2 * i] < iv[2 * (i - 1) + 1]) {
      set_error("vqx_adam_step_wn: updated ranges overlap at element %lld", (long long)iv[2 * i]);
      return -1;
    }
  if (covered != n) { set_error("vqx_adam_step_wn: rows + segments cover %lld of %lld elements", (long long)covered, (long long)n); return -1; }
  const int grid = P.row_off[n_layers] + P.seg_blk[n_segs];
  if (grid > 0)
    hipLaunchKernelGGL(adam_wn_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, p, g, m, v, hyper, sumsq,
                       max_norm, rows_dev, segs_dev, P);
  return launch_status("vqx_adam_step_wn");
}

extern "C" int vqx_radam_hyper(int64_t* step, double lr0, double gamma, int32_t step_size, double beta1,
                               double beta2, double eps, float* hyper, vqx_stream_t stream) {
  if (step_size < 1) { set_error("vqx_radam_hyper: step_size < 1"); return -1; }
  if (!(beta2 > 0.0 && beta2 < 1.0) || !step || !hyper) { set_error("vqx_radam_hyper: bad arguments"); return -1; }
  hipLaunchKernelGGL(radam_hyper_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, step, lr0, gamma, step_size, beta1,
                     beta2, eps, hyper);
  return launch_status("vqx_radam_hyper");
}

extern "C" int vqx_radam_step(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper,
                              const float* sumsq, float max_norm, vqx_stream_t stream) {
  if (n <= 0) return 0;
  if (!p || !g || !m || !v || !hyper) { set_error("vqx_radam_step: null pointer"); return -1; }
  hipLaunchKernelGGL(radam_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n,
                     hyper, sumsq, max_norm);
  return launch_status("vqx_radam_step");
}

// the 8-element chunk path when the shapes allow it (see map8_kernel); false: not taken
static bool map8_launch(const void* src, int32_t lds, int32_t sdt, void* dst, int32_t ldd, int32_t ddt, int64_t rows,
                        int32_t cols, float scale, int32_t act, hipStream_t s, void* zdst = nullptr, int32_t ldz = 0,
                        int64_t zrows = 0, int32_t zcols = 0) {
  if (cols % 8 || ldd % 8 || (src && lds % 8) || (rows * cols + zrows * zcols) / 8 >= (int64_t)1 << 31 ||
      ((uintptr_t)dst & 15) || ((uintptr_t)src & 15) || (zdst && (zcols % 8 || ldz % 8 || ((uintptr_t)zdst & 15))))
    return false;
  const int n8 = (int)(rows * cols / 8), cpr = cols / 8;
  const int n8z = zdst ? (int)(zrows * zcols / 8) : 0, cprz = zdst ? zcols / 8 : 1;
  const int grid = grid_for(n8 + n8z, 256, 2048);
  const bool sb = sdt == VQX_BF16, db = ddt == VQX_BF16;
  if (!src) {
    if (db) hipLaunchKernelGGL((map8_kernel<float, bf16_t, true>), dim3(grid), dim3(256), 0, s, nullptr, 0, (bf16_t*)dst, ldd, n8, cpr, 1.f, 0, (bf16_t*)zdst, ldz, n8z, cprz);
    else hipLaunchKernelGGL((map8_kernel<float, float, true>), dim3(grid), dim3(256), 0, s, nullptr, 0, (float*)dst, ldd, n8, cpr, 1.f, 0, (float*)zdst, ldz, n8z, cprz);
  } else if (sb && db) {
    hipLaunchKernelGGL((map8_kernel<bf16_t, bf16_t, false>), dim3(grid), dim3(256), 0, s, (const bf16_t*)src, lds, (bf16_t*)dst, ldd, n8, cpr, scale, act, (bf16_t*)zdst, ldz, n8z, cprz);
  } else if (sb) {
    hipLaunchKernelGGL((map8_kernel<bf16_t, float, false>), dim3(grid), dim3(256), 0, s, (const bf16_t*)src, lds, (float*)dst, ldd, n8, cpr, scale, act, (float*)zdst, ldz, n8z, cprz);
  } else if (db) {
    hipLaunchKernelGGL((map8_kernel<float, bf16_t, false>), dim3(grid), dim3(256), 0, s, (const float*)src, lds, (bf16_t*)dst, ldd, n8, cpr, scale, act, (bf16_t*)zdst, ldz, n8z, cprz);
  } else {
    hipLaunchKernelGGL((map8_kernel<float, float, false>), dim3(grid), dim3(256), 0, s, (const float*)src, lds, (float*)dst, ldd, n8, cpr, scale, act, (float*)zdst, ldz, n8z, cprz);
  }
  return true;
}

extern "C" int vqx_convert_2d(const void* src, int32_t ld_src, int32_t src_dtype, void* dst, int32_t ld_dst,
                              int32_t dst_dtype, int64_t rows, int32_t cols, vqx_stream_t stream) {
  if (rows <= 0 || cols <= 0) return 0;
  if (!dst) { set_error("vqx_convert_2d: null dst"); return -1; }
  if (map8_launch(src, ld_src, src_dtype, dst, ld_dst, dst_dtype, rows, cols, 1.f, VQX_PRO_NONE, (hipStream_t)stream))
    return launch_status("vqx_convert_2d");
  hipLaunchKernelGGL(convert_2d_kernel, dim3(grid_for(rows * cols, 256, 8192)), dim3(256), 0, (hipStream_t)stream,
                     src, ld_src, src_dtype, dst, ld_dst, dst_dtype, rows, cols);
  return launch_status("vqx_convert_2d");
}

extern "C" int vqx_convert_2d_zero2(const void* src, int32_t ld_src, int32_t src_dtype, void* dst, int32_t ld_dst,
                                    int32_t dst_dtype, int64_t rows, int32_t cols, void* zero_dst, int32_t ld_zero,
                                    int64_t zero_rows, int32_t zero_cols, vqx_stream_t stream) {
  if (rows <= 0 || cols <= 0 || zero_rows < 0 || zero_cols < 0) { set_error("vqx_convert_2d_zero2: bad shape"); return -1; }
  if (!dst || (!zero_dst && zero_rows * zero_cols)) { set_error("vqx_convert_2d_zero2: null dst"); return -1; }
  hipStream_t s = (hipStream_t)stream;
  if (map8_launch(src, ld_src, src_dtype, dst, ld_dst, dst_dtype, rows, cols, 1.f, VQX_PRO_NONE, s, zero_dst, ld_zero,
                  zero_rows, zero_cols))
    return launch_status("vqx_convert_2d_zero2");
  // unaligned shapes: the two element passes
  const int rc1 = vqx_convert_2d(src, ld_src, src_dtype, dst, ld_dst, dst_dtype, rows, cols, stream);
  if (rc1 || !zero_rows || !zero_cols) return rc1;
  return vqx_convert_2d(nullptr, 0, 0, zero_dst, ld_zero, dst_dtype, zero_rows, zero_cols, stream);
}

extern "C" int vqx_scale_act_2d(const void* src, int32_t ld_src, int32_t src_dtype, void* dst, int32_t ld_dst,
                                int32_t dst_dtype, int64_t rows, int32_t cols, float scale, int32_t act,
                                vqx_stream_t stream) {
  if (rows <= 0 || cols <= 0) return 0;
  if (!dst || !src) { set_error("vqx_scale_act_2d: null pointer"); return -1; }
  if (map8_launch(src, ld_src, src_dtype, dst, ld_dst, dst_dtype, rows, cols, scale, act, (hipStream_t)stream))
    return launch_status("vqx_scale_act_2d");
  hipLaunchKernelGGL(scale_act_2d_kernel, dim3(grid_for(rows * cols, 256, 8192)), dim3(256), 0, (hipStream_t)stream,
                     src, ld_src, src_dtype, dst, ld_dst, dst_dtype, rows, cols, scale, act);
  return launch_status("vqx_scale_act_2d");
}

extern "C" int vqx_linear_batched_fwd(const vqx_linear_layer* table_dev, int32_t n, const float* c, int32_t B,
                                      int32_t I, int32_t O, vqx_stream_t stream) {
  if (!table_dev || n < 1 || !c || B < 1 || I < 1 || O < 1) { set_error("vqx_linear_batched_fwd: bad arguments"); return -1; }
  if (I == kCondI && O % kCondO == 0 && ((uintptr_t)c & 15) == 0)  // any B: 16-row tiles in turn
    hipLaunchKernelGGL(linear_cond_fwd_kernel, dim3(O / kCondO, n), dim3(256), 0, (hipStream_t)stream, table_dev, c,
                       (const int64_t*)nullptr, B, O);
  else
    hipLaunchKernelGGL(linear_batched_fwd_kernel, dim3((O + kLT - 1) / kLT, n, (B + kLT - 1) / kLT), dim3(256), 0,
                       (hipStream_t)stream, table_dev, c, B, I, O);
  return launch_status("vqx_linear_batched_fwd");
}

extern "C" int vqx_linear_batched_bwd(const vqx_linear_layer* table_dev, int32_t n, const float* c, int32_t B,
                                      int32_t I, int32_t O, float* dc, float* partials, vqx_stream_t stream) {
  if (!table_dev || n < 1 || !c || B < 1 || I < 1 || O < 1) { set_error("vqx_linear_batched_bwd: bad arguments"); return -1; }
  if (dc && !partials) { set_error("vqx_linear_batched_bwd: dc needs partials [n*ceil(O/64)][B][I]"); return -1; }
  hipStream_t s = (hipStream_t)stream;
  const int nO = (O + kLT - 1) / kLT;
  if (I == kCondI && B <= kCondB && O % kCondO == 0 && ((uintptr_t)c & 15) == 0)
    hipLaunchKernelGGL(linear_cond_bwd_w_kernel, dim3(O / kCondO, n), dim3(256), 0, s, table_dev, c,
                       (const int64_t*)nullptr, B, O);
  else
    hipLaunchKernelGGL(linear_batched_bwd_w_kernel, dim3(nO, n, (I + kLT - 1) / kLT), dim3(256), 0, s,
                       table_dev, c, B, I, O);
  if (dc) {
    // any B (16-row tiles in turn), nO slices per layer as the tiled kernel: a row's dc does not depend on B
    if (I == kCondI && O % kCondO == 0 && kCondO == kLT)
      hipLaunchKernelGGL(linear_cond_bwd_x_kernel, dim3(O / kCondO, n), dim3(256), 0, s, table_dev, B, O, partials);
    else
      hipLaunchKernelGGL(linear_batched_bwd_x_kernel, dim3(nO, n, ((B + kLT - 1) / kLT) * ((I + kLT - 1) / kLT)),
                         dim3(256), 0, s, table_dev, B, I, O, partials);
    const int64_t ne = (int64_t)B * I;
    hipLaunchKernelGGL(sum_slices_wide_kernel, dim3((unsigned)((ne + 63) / 64)), dim3(256), 0, s, partials, n * nO, ne,
                       dc);
  }
  return launch_status("vqx_linear_batched_bwd");
}

static bool linear_ids_ok(const vqx_linear_layer* t, int n, const float* emb, const int64_t* ids, int B, int I, int O,
                          const char* who) {
  if (!t || n < 1 || !emb || !ids || B < 1 || B > kCondB || I != kCondI || O % kCondO || ((uintptr_t)emb & 15)) {
    set_error("%s: needs I = %d, 1 <= B <= %d, O %% %d == 0 and a 16-B aligned table", who, kCondI, kCondB, kCondO);
    return false;
  }
  return true;
}

extern "C" int vqx_linear_batched_fwd_ids(const vqx_linear_layer* table_dev, int32_t n, const float* emb,
                                          const int64_t* ids, int32_t B, int32_t I, int32_t O, vqx_stream_t stream) {
  if (!linear_ids_ok(table_dev, n, emb, ids, B, I, O, "vqx_linear_batched_fwd_ids")) return -1;
  hipLaunchKernelGGL(linear_cond_fwd_kernel, dim3(O / kCondO, n), dim3(256), 0, (hipStream_t)stream, table_dev, emb, ids,
                     B, O);
  return launch_status("vqx_linear_batched_fwd_ids");
}

extern "C" int vqx_step_prologue(const vqx_wn_layer* wn_host, const vqx_wn_layer* wn_dev, int32_t n_wn,
                                 const vqx_linear_layer* cond_table_dev, int32_t n_cond, const float* emb,
                                 const int64_t* ids, int32_t B, int32_t I, int32_t O, const float* x_nct, int32_t xB,
                                 int32_t C, int32_t T, void* y, int32_t ldy, int32_t y_dtype, vqx_stream_t stream) {
  WnUnits U;
  U.n = 0;
  U.off[0] = 0;
  if (n_wn < 0 || n_wn > kWnMaxL || (n_wn && (!wn_host || !wn_dev))) { set_error("vqx_step_prologue: 0 <= n_wn <= %d layers with both tables", kWnMaxL); return -1; }
  if (n_wn) {
    if (wn_fwd_check(wn_host, n_wn, "vqx_step_prologue") < 0) return -1;
    U.n = n_wn;
    for (int i = 0; i < n_wn; ++i) U.off[i + 1] = U.off[i] + wn_pack_units(wn_host[i]);
  }
  if (n_cond < 0 || (n_cond && !linear_ids_ok(cond_table_dev, n_cond, emb, ids, B, I, O, "vqx_step_prologue"))) return -1;
  if (x_nct && (xB < 1 || C < 1 || T < 1 || !y || ldy < C || (y_dtype != VQX_F32 && y_dtype != VQX_BF16))) { set_error("vqx_step_prologue: bad transpose arguments"); return -1; }
  const int cond_bx = n_cond ? O / kCondO : 1, n_cond_blocks = n_cond * (n_cond ? O / kCondO : 0);
  const int tx_bx = x_nct ? (T + 31) / 32 : 1, tx_by = x_nct ? (C + 31) / 32 : 1;
  const int64_t n_tx = x_nct ? (int64_t)tx_bx * tx_by * xB : 0;
  const int64_t grid = n_cond_blocks + n_tx + U.off[U.n];
  if (grid > INT32_MAX) { set_error("vqx_step_prologue: grid too large"); return -1; }
  if (grid == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (y_dtype == VQX_BF16)
    hipLaunchKernelGGL(step_prologue_kernel<bf16_t>, dim3((unsigned)grid), dim3(256), 0, s, wn_dev, U, cond_table_dev,
                       n_cond_blocks, cond_bx, emb, ids, B, O, x_nct, C, T, tx_bx, tx_by, (int)n_tx, (bf16_t*)y, ldy);
  else
    hipLaunchKernelGGL(step_prologue_kernel<float>, dim3((unsigned)grid), dim3(256), 0, s, wn_dev, U, cond_table_dev,
                       n_cond_blocks, cond_bx, emb, ids, B, O, x_nct, C, T, tx_bx, tx_by, (int)n_tx, (float*)y, ldy);
  return launch_status("vqx_step_prologue");
}

extern "C" int vqx_linear_batched_bwd_ids(const vqx_linear_layer* table_dev, int32_t n, const float* emb,
                                          const int64_t* ids, int32_t B, int32_t I, int32_t O, float* dc,
                                          float* partials, vqx_stream_t stream) {
  if (!linear_ids_ok(table_dev, n, emb, ids, B, I, O, "vqx_linear_batched_bwd_ids")) return -1;
  if (dc && !partials) { set_error("vqx_linear_batched_bwd_ids: dc needs partials [n*O/64][B][I]"); return -1; }
  hipStream_t s = (hipStream_t)stream;
  if (!dc || 2 * (int64_t)n > 65535) {  // (grid y: 2n)
    hipLaunchKernelGGL(linear_cond_bwd_w_kernel, dim3(O / kCondO, n), dim3(256), 0, s, table_dev, emb, ids, B, O);
    if (dc)
      hipLaunchKernelGGL(linear_cond_bwd_x_kernel, dim3(O / kCondO, n), dim3(256), 0, s, table_dev, B, O, partials);
  } else {  // the weight and data gradients in one grid (round 6: two launches)
    hipLaunchKernelGGL(linear_cond_bwd_kernel, dim3(O / kCondO, 2 * n), dim3(256), 0, s, table_dev, emb, ids, B, O, n,
                       partials);
  }
  if (dc) {
    const int64_t ne = (int64_t)B * I;
    hipLaunchKernelGGL(sum_slices_wide_kernel, dim3((unsigned)((ne + 63) / 64)), dim3(256), 0, s, partials,
                       n * (O / kCondO), ne, dc);
  }
  return launch_status("vqx_linear_batched_bwd_ids");
}

extern "C" int vqx_gn_finalize_tiles(const float* parts, int64_t n_rows, int32_t T, int32_t C, int32_t G, float eps,
                                     float* mean_rstd, vqx_stream_t stream) {
  if (!parts || !mean_rstd || T % 128 || n_rows % T || G < 1 || C % G || (C / G) % 128) {
    set_error("vqx_gn_finalize_tiles: needs T %% 128 == 0 and C/G %% 128 == 0");
    return -1;
  }
  const int B = (int)(n_rows / T);
  hipLaunchKernelGGL(gn_finalize_tiles_kernel, dim3((B * G + 127) / 128), dim3(128), 0, (hipStream_t)stream, parts, B,
                     G, T / 128, C / 128, (C / G) / 128, eps, mean_rstd);
  return launch_status("vqx_gn_finalize_tiles");
}
