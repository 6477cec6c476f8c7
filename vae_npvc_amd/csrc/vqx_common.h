// Shared device helpers for libvqx (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/vqx.h"

typedef unsigned short bf16_t;  // storage type of bf16 activations/weights
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

#define VQX_LDS(T) __attribute__((address_space(3))) T

namespace vqx {

void set_error(const char* fmt, ...);
int launch_status(const char* what);

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32: round-to-nearest-even, NaN-preserving
  return *reinterpret_cast<bf16_t*>(&b);
}

// two floats -> packed bf16 pair (lo in bits 0-15): one v_cvt_pk_bf16_f32
// (round-to-nearest-even) instead of two conversions plus shift and or
__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
  const f2_t v = {lo, hi};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, b2_t));
}

template <typename T> struct Elem;
template <> struct Elem<float> {
  __device__ static __forceinline__ float ld(const void* p, int64_t i) { return ((const float*)p)[i]; }
  __device__ static __forceinline__ void st(void* p, int64_t i, float v) { ((float*)p)[i] = v; }
};
template <> struct Elem<bf16_t> {
  __device__ static __forceinline__ float ld(const void* p, int64_t i) { return bf2f(((const bf16_t*)p)[i]); }
  __device__ static __forceinline__ void st(void* p, int64_t i, float v) { ((bf16_t*)p)[i] = f2bf(v); }
};

__device__ __forceinline__ float ld_dt(const void* p, int64_t i, int dt) {
  return dt == VQX_BF16 ? bf2f(((const bf16_t*)p)[i]) : ((const float*)p)[i];
}
__device__ __forceinline__ void st_dt(void* p, int64_t i, float v, int dt) {
  if (dt == VQX_BF16) ((bf16_t*)p)[i] = f2bf(v); else ((float*)p)[i] = v;
}

// GLU activations with the hardware reciprocal (v_rcp_f32, 1 ulp) instead of
// IEEE division (a ~10-instruction scale/fixup sequence): the GroupNorm/GLU
// kernels that call these per element are VALU-bound, not HBM-bound.
#ifndef VQX_FAST_RCP
#define VQX_FAST_RCP 1
#endif
// FAST = false keeps the IEEE division: the fp32 compute mode is the parity
// mode (smoke() and the golden-step tests compare it with the fp32 oracle),
// so only the bf16 instantiations take the hardware reciprocal.
template <bool FAST = true>
__device__ __forceinline__ float frcp(float x) {
  if constexpr (FAST && VQX_FAST_RCP) return __builtin_amdgcn_rcpf(x);
  else return 1.f / x;
}
template <bool FAST = true>
__device__ __forceinline__ float fsigmoid(float x) { return frcp<FAST>(1.f + __expf(-x)); }
template <bool FAST = true>
__device__ __forceinline__ float ftanh(float x) { return 2.f * frcp<FAST>(1.f + __expf(-2.f * x)) - 1.f; }

// Chan et al. parallel merge of (count, mean, M2) moments: a <- a (+) b.
__device__ __forceinline__ void moments_merge(float& na, float& ma, float& qa, float nb, float mb, float qb) {
  const float n = na + nb;
  if (nb == 0.f) return;
  const float d = mb - ma;
  const float f = nb / n;  // exact: GroupNorm statistics feed the parity checks
  ma = fmaf(d, f, ma);
  qa = qa + qb + d * d * na * f;
  na = n;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum (blockDim.x multiple of 64, <= 1024); result valid in all threads.
__device__ __forceinline__ float block_sum(float v, float* scratch /* >= 16 floats */) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += scratch[i];  // fixed order: deterministic
  return s;
}

// N block sums at once (one pair of barriers): each value's waves added in
// wave order, as block_sum does
template <int N>
__device__ __forceinline__ void block_sum_n(float (&v)[N], float (*scratch)[16]) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] = wave_sum(v[k]);
  __syncthreads();
  if (l == 0) {
#pragma unroll
    for (int k = 0; k < N; ++k) scratch[k][w] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k) {
    float t = 0.f;
    for (int i = 0; i < nw; ++i) t += scratch[k][i];
    v[k] = t;
  }
}

// N block sums as a block of NV * blockDim.x threads computes them with
// block_sum_n (the same bits): thread t holds the values of virtual threads
// t + j*blockDim.x (j < NV), whose virtual wave is w + j*waves; the virtual
// waves' sums are added in order.  NV * waves <= 16.
template <int N, int NV>
__device__ __forceinline__ void block_sum_nv(float (&v)[N][NV], float (*scratch)[16], float (&out)[N]) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < N; ++k)
#pragma unroll
    for (int j = 0; j < NV; ++j) v[k][j] = wave_sum(v[k][j]);
  __syncthreads();
  if (l == 0) {
#pragma unroll
    for (int k = 0; k < N; ++k)
#pragma unroll
      for (int j = 0; j < NV; ++j) scratch[k][w + j * nw] = v[k][j];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k) {
    float t = 0.f;
    for (int i = 0; i < nw * NV; ++i) t += scratch[k][i];
    out[k] = t;
  }
}

// Last-arriver hand-off between the workgroups of one launch (MI355X_MICROARCH.md
// "inter-workgroup visibility", table row 1): every workgroup stores the words
// it hands off with st_agent (sc1 stores), then calls arrive_last: each wave
// waits for its stores, the barrier joins them, one lane adds to the
// agent-scope counter, and the workgroup whose add returned n-1 (told to its
// waves through LDS) gets true, resets the counter for the next launch and
// reads the words with ld_agent (sc1 loads).  No workgroup waits for another.
__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool arrive_last(unsigned* counter, unsigned n) {
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == n - 1;
    if (old == n - 1) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return last != 0;
}

// Bijective XCD-aware remap of a linear block id (guide §5 "XCD swizzle must
// be bijective"): blocks b and b+8 share an XCD, so give each XCD group a
// contiguous range of logical tiles.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

}  // namespace vqx
