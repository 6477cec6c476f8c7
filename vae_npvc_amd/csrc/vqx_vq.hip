// EMA vector quantizer kernels (layers_vq.py:166-334) for gfx950.
//
// vq_forward: one launch does distance -> argmin -> gather -> commitment
// partial sums -> EMA scatter statistics, reading z in its frame-major
// layout (no transpose copy, layers_vq.py:274-276) and never materialising
// the (N, K) distance matrix (layers_vq.py:285-289).
//
// Geometry: 4 waves x 16 frames per workgroup.  Each wave keeps its 16x128
// f32 z block in registers as the A operand of v_mfma_f32_16x16x4_f32; the
// codebook streams through LDS in 64-code tiles (double-buffered, XOR-
// swizzled 16-B chunks so the ds_read_b128 B-fragment reads are
// conflict-free).  Dot products are exact f32 (fmaf chains), the distance
// is formed in the reference's order (||z||^2 + ||e||^2) - 2 z.e, and the
// argmin keeps the first minimum (strict '<' in ascending code order, then
// a lowest-index tie-break across lanes), matching torch.argmin.
#include "vqx_common.h"

namespace vqx {

constexpr int VQ_D = 128;
constexpr int VQ_TILE = 64;                 // codes per LDS tile
constexpr int VQ_TILE_BYTES = VQ_TILE * VQ_D * 4;

__global__ __launch_bounds__(256) void vq_forward_kernel(const float* __restrict__ z, int64_t N,
                                                         const float* __restrict__ E, int K,
                                                         int64_t* __restrict__ idx_out,
                                                         float* __restrict__ zq, void* __restrict__ zq_c,
                                                         int zq_dt, float* __restrict__ partials,
                                                         float* __restrict__ bsum, float* __restrict__ bcnt) {
  __shared__ __attribute__((aligned(16))) char smem[2 * VQ_TILE_BYTES];
  __shared__ float ee_lds[2][VQ_TILE];
  __shared__ float red[16];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int q = lane >> 4, j16 = lane & 15;
  const int64_t row0 = (int64_t)blockIdx.x * 64 + w * 16;
  const int64_t my_row = row0 + j16;  // A-operand row of this lane
  const bool row_ok = my_row < N;

  // z fragments: zf[kb] = z[my_row][16kb + 4q .. +3]
  f32x4_t zf[8];
  float zz = 0.f;
#pragma unroll
  for (int kb = 0; kb < 8; ++kb) {
    f32x4_t v = {0.f, 0.f, 0.f, 0.f};
    if (row_ok) v = *(const f32x4_t*)(z + my_row * VQ_D + 16 * kb + 4 * q);
    zf[kb] = v;
    zz = fmaf(v[0], v[0], zz);
    zz = fmaf(v[1], v[1], zz);
    zz = fmaf(v[2], v[2], zz);
    zz = fmaf(v[3], v[3], zz);
  }
  zz += __shfl_xor(zz, 16, 64);
  zz += __shfl_xor(zz, 32, 64);
  // C layout of 16x16x4: lane holds rows 4q+r (r=0..3), code column j16.
  float zz_r[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) zz_r[r] = __shfl(zz, 4 * q + r, 64);

  float best_d[4];
  int best_i[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { best_d[r] = INFINITY; best_i[r] = 0x7fffffff; }

  const int ntiles = (K + VQ_TILE - 1) / VQ_TILE;
  f32x4_t stage[8];
  auto load_tile = [&](int t) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = tid + 256 * i;        // chunk id in tile: code c>>5, chunk c&31
      const int code = t * VQ_TILE + (c >> 5);
      f32x4_t v = {0.f, 0.f, 0.f, 0.f};
      if (code < K) v = *(const f32x4_t*)(E + (int64_t)code * VQ_D + 4 * (c & 31));
      stage[i] = v;
    }
  };
  auto store_tile = [&](int buf) {
    char* base = smem + buf * VQ_TILE_BYTES;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = tid + 256 * i;
      const int code = c >> 5, ch = c & 31;
      *(f32x4_t*)(base + code * 512 + 16 * (ch ^ (code & 15))) = stage[i];
    }
  };
  auto ee_tile = [&](int buf, int t) {
    // 4 threads per code, 32 elements each, read back from LDS
    const char* base = smem + buf * VQ_TILE_BYTES;
    const int code = tid >> 2, part = tid & 3;
    float s = 0.f;
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) {
      const int ch = part * 8 + cc;
      f32x4_t v = *(const f32x4_t*)(base + code * 512 + 16 * (ch ^ (code & 15)));
      s = fmaf(v[0], v[0], s); s = fmaf(v[1], v[1], s); s = fmaf(v[2], v[2], s); s = fmaf(v[3], v[3], s);
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (part == 0) ee_lds[buf][code] = s;
    (void)t;
  };

  load_tile(0);
  store_tile(0);
  __syncthreads();
  ee_tile(0, 0);
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    const bool more = (t + 1) < ntiles;
    if (more) load_tile(t + 1);
    const char* base = smem + buf * VQ_TILE_BYTES;
#pragma unroll
    for (int cb = 0; cb < VQ_TILE / 16; cb += 2) {
      f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      const int c0 = cb * 16 + j16, c1 = c0 + 16;
#pragma unroll
      for (int kb = 0; kb < 8; ++kb) {
        const int ch = 4 * kb + q;
        f32x4_t b0 = *(const f32x4_t*)(base + c0 * 512 + 16 * (ch ^ (c0 & 15)));
        f32x4_t b1 = *(const f32x4_t*)(base + c1 * 512 + 16 * (ch ^ (c1 & 15)));
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(zf[kb][m], b0[m], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(zf[kb][m], b1[m], acc1, 0, 0, 0);
        }
      }
      const int code0 = t * VQ_TILE + c0, code1 = code0 + 16;
      const float e0 = ee_lds[buf][c0], e1 = ee_lds[buf][c1];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (code0 < K) {
          const float d0 = __fsub_rn(__fadd_rn(zz_r[r], e0), __fmul_rn(2.f, acc0[r]));
          if (d0 < best_d[r]) { best_d[r] = d0; best_i[r] = code0; }
        }
        if (code1 < K) {
          const float d1 = __fsub_rn(__fadd_rn(zz_r[r], e1), __fmul_rn(2.f, acc1[r]));
          if (d1 < best_d[r]) { best_d[r] = d1; best_i[r] = code1; }
        }
      }
    }
    if (more) {
      store_tile(buf ^ 1);
      __syncthreads();
      ee_tile(buf ^ 1, t + 1);
    }
    __syncthreads();
  }

  // argmin across the 16 lanes of each row group (lowest index on ties)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      const float od = __shfl_xor(best_d[r], o, 64);
      const int oi = __shfl_xor(best_i[r], o, 64);
      if (od < best_d[r] || (od == best_d[r] && oi < best_i[r])) { best_d[r] = od; best_i[r] = oi; }
    }
  }
  // NaN rows (all comparisons false) fall back to code 0 like torch.argmin's
  // first-element seed would not; keep them well-defined.
  // idx of this lane's A-row j16: held by group j16>>2, register j16&3.
  int my_idx = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int v = __shfl(best_i[r], 16 * (j16 >> 2), 64);
    if ((j16 & 3) == r) my_idx = v;
  }
  if (my_idx >= K || my_idx < 0) my_idx = 0;

  float sq = 0.f;
  if (row_ok) {
    if (q == 0) idx_out[my_row] = my_idx;
#pragma unroll
    for (int kb = 0; kb < 8; ++kb) {
      const int d0 = 16 * kb + 4 * q;
      const f32x4_t e = *(const f32x4_t*)(E + (int64_t)my_idx * VQ_D + d0);
      if (zq) *(f32x4_t*)(zq + my_row * VQ_D + d0) = e;
      if (zq_c) {
        if (zq_dt == VQX_BF16) {
          bf16_t* o = (bf16_t*)zq_c + my_row * VQ_D + d0;
          uint2 pk;
          pk.x = pack_bf16x2(e[0], e[1]);
          pk.y = pack_bf16x2(e[2], e[3]);
          *(uint2*)o = pk;
        } else {
          *(f32x4_t*)((float*)zq_c + my_row * VQ_D + d0) = e;
        }
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const float df = __fsub_rn(e[m], zf[kb][m]);
        sq = fmaf(df, df, sq);
      }
    }
  }

  // ---- EMA statistics: per-code sums of z over this workgroup's 64 frames.
  // Sort the (code, frame) pairs with a wave-wide bitonic network, then each
  // thread walks a run of the sorted frames for one dimension d and flushes a
  // partial sum per code segment: one contiguous 256-B atomic wave-instruction
  // per (segment, 64 dims) instead of one scattered atomic per element, and no
  // same-address pile-up when the codebook usage is concentrated.
  if (bsum) {
    float* zl = (float*)smem;                       // [64][128] frame block (tile buffers are free now)
    int* codes = (int*)(smem + 64 * VQ_D * 4);      // [64] code per local frame (K = invalid)
    int* order = codes + 64;                        // [64] frames sorted by code
#pragma unroll
    for (int kb = 0; kb < 8; ++kb) *(f32x4_t*)(zl + (w * 16 + j16) * VQ_D + 16 * kb + 4 * q) = zf[kb];
    if (q == 0) codes[w * 16 + j16] = row_ok ? my_idx : K;
    __syncthreads();
    if (w == 0) {
      int key = codes[lane] * 64 + lane;
#pragma unroll
      for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
          const int other = __shfl_xor(key, j, 64);
          const bool up = (lane & k) == 0, lower = (lane & j) == 0;
          key = (lower == up) ? min(key, other) : max(key, other);
        }
      }
      order[lane] = key & 63;
    }
    __syncthreads();
    const int d = tid & 127, half = tid >> 7;
    int cur = -1, cnt = 0;
    float acc = 0.f;
    for (int p = 32 * half; p < 32 * half + 32; ++p) {
      const int r = order[p];
      const int c = codes[r];
      if (c != cur) {
        if (cur >= 0 && cur < K) {
          atomicAdd(bsum + (int64_t)cur * VQ_D + d, acc);
          if (d == 0 && bcnt) atomicAdd(bcnt + cur, (float)cnt);
        }
        cur = c;
        acc = 0.f;
        cnt = 0;
      }
      acc += zl[r * VQ_D + d];
      ++cnt;
    }
    if (cur >= 0 && cur < K) {
      atomicAdd(bsum + (int64_t)cur * VQ_D + d, acc);
      if (d == 0 && bcnt) atomicAdd(bcnt + cur, (float)cnt);
    }
  }
  const float tot = block_sum(sq, red);
  if (tid == 0) partials[blockIdx.x] = tot;
}

// Deterministic single-workgroup sum of n partials into out[0] (optionally scaled).
__global__ void sum_partials_kernel(const float* __restrict__ p, int n, float scale, float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += p[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[0] = s * scale;
}

// EMA codebook update, one workgroup (layers_vq.py:203-233).
// EMA update in two launches: the K*D elementwise update over many workgroups
// (one exact division per element; a single workgroup took ~48 us), each
// writing its squared-difference partial; then one workgroup for the per-code
// terms, the emb_elem update and the diagnostics, summing the partials in a
// fixed order (deterministic).
constexpr int kEmaElems = 1024;  // elements per workgroup of vq_ema_elem_kernel

__global__ __launch_bounds__(256) void vq_ema_elem_kernel(float* __restrict__ emb_sum,
                                                          const float* __restrict__ emb_elem, float* __restrict__ E,
                                                          const float* __restrict__ bsum,
                                                          const float* __restrict__ bcnt,
                                                          const float* __restrict__ rand_rows, int K, int D, float mu,
                                                          float one_minus_mu, float thr, float* __restrict__ part) {
  __shared__ float red[16];
  const int i0 = blockIdx.x * kEmaElems;
  float dsq = 0.f;
  for (int i = i0 + threadIdx.x; i < min(K * D, i0 + kEmaElems); i += blockDim.x) {
    const int k = i / D;
    const float s = __fadd_rn(__fmul_rn(mu, emb_sum[i]), __fmul_rn(one_minus_mu, bsum[i]));
    const float el = __fadd_rn(__fmul_rn(mu, emb_elem[k]), __fmul_rn(one_minus_mu, bcnt[k]));
    emb_sum[i] = s;
    const float u = (el >= thr) ? 1.f : 0.f;
    // usage*(sum/elem) + (1-usage)*rand, evaluated like the reference
    const float newe = __fadd_rn(__fmul_rn(u, __fdiv_rn(s, el)), __fmul_rn(1.f - u, rand_rows[i]));
    const float diff = __fsub_rn(newe, E[i]);
    dsq = fmaf(diff, diff, dsq);
    E[i] = newe;
  }
  dsq = block_sum(dsq, red);
  if (threadIdx.x == 0) part[blockIdx.x] = dsq;
}

__global__ __launch_bounds__(1024) void vq_ema_final_kernel(float* __restrict__ emb_elem,
                                                            const float* __restrict__ bcnt, int K, int D, float mu,
                                                            float one_minus_mu, float thr,
                                                            const float* __restrict__ part, int nparts,
                                                            float* __restrict__ diag) {
  __shared__ float red[16];
  float dsq = 0.f;
  for (int b = threadIdx.x; b < nparts; b += blockDim.x) dsq += part[b];
  dsq = block_sum(dsq, red);
  __syncthreads();
  float total = 0.f;
  for (int k = threadIdx.x; k < K; k += blockDim.x) total += bcnt[k];
  total = block_sum(total, red);
  __syncthreads();
  float ent = 0.f, used = 0.f, usage = 0.f;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const float c = bcnt[k];
    const float p = c / total;
    ent += p * logf(p + 1e-8f);
    used += (c >= thr) ? 1.f : 0.f;
    const float el = __fadd_rn(__fmul_rn(mu, emb_elem[k]), __fmul_rn(one_minus_mu, c));
    usage += (el >= thr) ? 1.f : 0.f;
  }
  __syncthreads();
  ent = block_sum(ent, red);
  __syncthreads();
  used = block_sum(used, red);
  __syncthreads();
  usage = block_sum(usage, red);
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += blockDim.x)
    emb_elem[k] = __fadd_rn(__fmul_rn(mu, emb_elem[k]), __fmul_rn(one_minus_mu, bcnt[k]));
  if (threadIdx.x == 0) {
    diag[0] = expf(-ent);
    diag[1] = used;
    diag[2] = usage;
    diag[3] = sqrtf(dsq) / sqrtf((float)K * (float)D);
  }
}

__global__ void gather_rows_kernel(const float* __restrict__ src, int ld, const int64_t* __restrict__ rows,
                                   int n_out, int D, float* __restrict__ out) {
  const int i = blockIdx.x;
  if (i >= n_out) return;
  const int64_t r = rows[i];
  for (int d = threadIdx.x; d < D; d += blockDim.x) out[(int64_t)i * D + d] = (r >= 0) ? src[r * ld + d] : 0.f;
}

template <typename T>
__global__ void commit_bwd_kernel(const float* __restrict__ z, const float* __restrict__ zq, int64_t n, float scale,
                                  T* __restrict__ dz) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    Elem<T>::st(dz, i, scale * __fsub_rn(z[i], zq[i]));
}

}  // namespace vqx

using namespace vqx;

extern "C" int vqx_vq_forward(const float* z, int64_t n_rows, int32_t D, const float* E, int32_t K, int64_t* idx,
                              float* zq, void* zq_c, int32_t zq_c_dtype, float* sqerr_out, float* partials,
                              float* bsum, float* bcnt, vqx_stream_t stream) {
  if (D != VQ_D) { set_error("vqx_vq_forward: only D=128 supported (got %d)", D); return -1; }
  if (K <= 0 || K % 16) { set_error("vqx_vq_forward: K=%d must be a positive multiple of 16", K); return -1; }
  if (n_rows <= 0 || !z || !E || !idx || !partials) { set_error("vqx_vq_forward: bad arguments"); return -1; }
  if (((uintptr_t)z | (uintptr_t)E) & 15) { set_error("vqx_vq_forward: z/E must be 16-byte aligned"); return -1; }
  hipStream_t s = (hipStream_t)stream;
  const int grid = (int)((n_rows + 63) / 64);
  hipLaunchKernelGGL(vq_forward_kernel, dim3(grid), dim3(256), 0, s, z, n_rows, E, K, idx, zq, zq_c, zq_c_dtype,
                     partials, bsum, bcnt);
  if (sqerr_out) hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(1024), 0, s, partials, grid, 1.0f, sqerr_out);
  return launch_status("vqx_vq_forward");
}

extern "C" int vqx_vq_ema_update(float* emb_sum, float* emb_elem, float* E, const float* bsum, const float* bcnt,
                                 const float* rand_rows, int32_t K, int32_t D, float mu, float threshold, float* diag,
                                 float* partials, vqx_stream_t stream) {
  if (K <= 0 || D <= 0 || !partials) { set_error("vqx_vq_ema_update: bad K/D or no partials"); return -1; }
  const float omm = (float)(1.0 - (double)mu);  // (1. - mu) in double, as the reference's Python float
  const int nb = (K * D + kEmaElems - 1) / kEmaElems;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(vq_ema_elem_kernel, dim3(nb), dim3(256), 0, s, emb_sum, emb_elem, E, bsum, bcnt, rand_rows, K,
                     D, mu, omm, threshold, partials);
  hipLaunchKernelGGL(vq_ema_final_kernel, dim3(1), dim3(1024), 0, s, emb_elem, bcnt, K, D, mu, omm, threshold,
                     partials, nb, diag);
  return launch_status("vqx_vq_ema_update");
}

extern "C" int vqx_gather_rows(const float* src, int32_t ld_src, const int64_t* rows, int32_t n_out, int32_t D,
                               float* out, vqx_stream_t stream) {
  if (n_out <= 0 || D <= 0) { set_error("vqx_gather_rows: bad sizes"); return -1; }
  hipLaunchKernelGGL(gather_rows_kernel, dim3(n_out), dim3(128), 0, (hipStream_t)stream, src, ld_src, rows, n_out, D,
                     out);
  return launch_status("vqx_gather_rows");
}

extern "C" int vqx_vq_commit_bwd(const float* z, const float* zq, int64_t count, float scale, void* dz, int32_t dtype,
                                 vqx_stream_t stream) {
  if (count <= 0) return 0;
  const int grid = (int)std::min<int64_t>((count + 255) / 256, 4096);
  if (dtype == VQX_BF16)
    hipLaunchKernelGGL(commit_bwd_kernel<bf16_t>, dim3(grid), dim3(256), 0, (hipStream_t)stream, z, zq, count, scale,
                       (bf16_t*)dz);
  else
    hipLaunchKernelGGL(commit_bwd_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, z, zq, count, scale,
                       (float*)dz);
  return launch_status("vqx_vq_commit_bwd");
}

// ===================================================================
// Straight-through VectorQuantizer (use_ema: false; layers_vq.py:9-163,
// reduction 'frame_mean', target_norm 1.0).  One wave per 128-wide row.
// ===================================================================
namespace {

__device__ __forceinline__ float wave_sum64(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Blocks [0, ceil(K/4)) renormalise the codebook rows, the rest the frames.
//   codebook (embed_norm, layers_vq.py:28-33, then :99): E *= 1/||E|| in
//     place, embn = (1.0*E)/||E||, e_len = ||E|| (after the in-place step);
//   frames (:97): z_norm = (1.0*z)/||z||, z_len = ||z||, and the per-block
//     sum of (z_norm - z)^2 (normalisation loss, :125-126).
__global__ __launch_bounds__(256) void vq_normalize_kernel(const float* __restrict__ z, int64_t N, float* __restrict__ E,
                                                           int K, float* __restrict__ zn, float* __restrict__ zlen,
                                                           float* __restrict__ embn, float* __restrict__ elen,
                                                           float* __restrict__ part) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kb = (K + 3) / 4;
  __shared__ float red[4];
  if ((int)blockIdx.x < kb) {
    const int k = blockIdx.x * 4 + w;
    if (k >= K) return;
    float2 e = *(const float2*)(E + (int64_t)k * 128 + 2 * lane);
    const float n1 = sqrtf(wave_sum64(e.x * e.x + e.y * e.y));
    const float f = 1.0f / n1;
    e.x *= f;
    e.y *= f;
    *(float2*)(E + (int64_t)k * 128 + 2 * lane) = e;
    const float n2 = sqrtf(wave_sum64(e.x * e.x + e.y * e.y));
    *(float2*)(embn + (int64_t)k * 128 + 2 * lane) = make_float2(e.x / n2, e.y / n2);
    if (lane == 0) elen[k] = n2;
    return;
  }
  const int64_t n = (int64_t)(blockIdx.x - kb) * 4 + w;
  float l = 0.f;
  if (n < N) {
    const float2 v = *(const float2*)(z + n * 128 + 2 * lane);
    const float nz = sqrtf(wave_sum64(v.x * v.x + v.y * v.y));
    const float2 u = make_float2(v.x / nz, v.y / nz);
    *(float2*)(zn + n * 128 + 2 * lane) = u;
    if (lane == 0) zlen[n] = nz;
    l = wave_sum64((u.x - v.x) * (u.x - v.x) + (u.y - v.y) * (u.y - v.y));
  }
  if (lane == 0) red[w] = l;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x - kb] = (red[0] + red[1]) + (red[2] + red[3]);
}

// perplexity exp(-sum p log(p + 1e-10)), p = counts / N (layers_vq.py:112-114)
__global__ __launch_bounds__(256) void vq_perplexity_kernel(const float* __restrict__ cnt, int K, float inv_n,
                                                            float* __restrict__ out) {
  __shared__ float red[16];
  float h = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) {
    const float p = cnt[k] * inv_n;
    h += p * logf(p + 1e-10f);
  }
  h = vqx::block_sum(h, red);
  if (threadIdx.x == 0) *out = expf(-h);
}

// Backward of  loss = x_loss + z_qut + beta * z_enc  through the quantizer.
// frames n: dzn = st(dzq_n) + beta*s*(zn - zq) [+ beta*s*(zn - z)]; with
//   normalisation dz = (dzn - zn (zn.dzn)) / ||z|| - beta*s*(zn - z), else
//   dz = dzn.  st(): the straight-through gradient from the decoder, zero on
//   frames the Jitter replaced (its copy comes from a detached tensor,
//   layers_vq.py:356,377).
// codes k: d = s*(cnt_k*emb_k - bsum_k) (= sum over the code's frames of
//   2(zq - zn)/(B*T), z_qut), then dE = (d - emb (emb.d)) / e_len through
//   emb = E/||E||, or dE = d without normalisation.
template <typename T>
__global__ __launch_bounds__(256) void vq_plain_bwd_kernel(const float* __restrict__ z, const float* __restrict__ zn,
                                                           const float* __restrict__ zlen, const float* __restrict__ zq,
                                                           const T* __restrict__ dzq, const int* __restrict__ src_t,
                                                           int Tn, int64_t N, int normalize, float beta, float s,
                                                           T* __restrict__ dz, const float* __restrict__ bsum,
                                                           const float* __restrict__ bcnt,
                                                           const float* __restrict__ emb, const float* __restrict__ elen,
                                                           int K, float* __restrict__ dE) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kb = (K + 3) / 4;
  if ((int)blockIdx.x < kb) {
    const int k = blockIdx.x * 4 + w;
    if (k >= K) return;
    const float2 e = *(const float2*)(emb + (int64_t)k * 128 + 2 * lane);
    const float2 b = *(const float2*)(bsum + (int64_t)k * 128 + 2 * lane);
    const float c = bcnt[k];
    float2 d = make_float2(s * (c * e.x - b.x), s * (c * e.y - b.y));
    if (normalize) {
      const float dot = wave_sum64(e.x * d.x + e.y * d.y);
      const float il = 1.0f / elen[k];
      d = make_float2((d.x - e.x * dot) * il, (d.y - e.y * dot) * il);
    }
    *(float2*)(dE + (int64_t)k * 128 + 2 * lane) = d;
    return;
  }
  const int64_t n = (int64_t)(blockIdx.x - kb) * 4 + w;
  if (n >= N) return;
  const int64_t o = n * 128 + 2 * lane;
  const float2 u = *(const float2*)(zn + o);
  const float2 q = *(const float2*)(zq + o);
  float g0 = 0.f, g1 = 0.f;
  const int t = (int)(n % Tn);
  if (dzq && (!src_t || src_t[t] == t)) {
    g0 = Elem<T>::ld(dzq, o);
    g1 = Elem<T>::ld(dzq, o + 1);
  }
  const float bs = beta * s;
  float d0 = g0 + bs * (u.x - q.x), d1 = g1 + bs * (u.y - q.y);
  if (normalize) {
    const float2 v = *(const float2*)(z + o);
    d0 += bs * (u.x - v.x);
    d1 += bs * (u.y - v.y);
    const float dot = wave_sum64(u.x * d0 + u.y * d1);
    const float il = 1.0f / zlen[n];
    d0 = (d0 - u.x * dot) * il - bs * (u.x - v.x);
    d1 = (d1 - u.y * dot) * il - bs * (u.y - v.y);
  }
  Elem<T>::st(dz, o, d0);
  Elem<T>::st(dz, o + 1, d1);
}

}  // namespace

extern "C" int vqx_vq_normalize(const float* z, int64_t n_rows, int32_t D, float* E, int32_t K, float* z_norm,
                                float* z_len, float* emb_norm, float* e_len, float* partials, float* normloss_out,
                                vqx_stream_t stream) {
  if (D != 128) { set_error("vqx_vq_normalize: z_dim must be 128"); return -1; }
  if (!z || !E || !z_norm || !z_len || !emb_norm || !e_len || !partials || n_rows < 1 || K < 1) {
    set_error("vqx_vq_normalize: bad arguments");
    return -1;
  }
  hipStream_t s = (hipStream_t)stream;
  const int kb = (K + 3) / 4;
  const int64_t zb = (n_rows + 3) / 4;
  hipLaunchKernelGGL(vq_normalize_kernel, dim3((unsigned)(kb + zb)), dim3(256), 0, s, z, n_rows, E, K, z_norm, z_len,
                     emb_norm, e_len, partials);
  if (normloss_out) hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(1024), 0, s, partials, (int)zb, 1.0f, normloss_out);
  return launch_status("vqx_vq_normalize");
}

extern "C" int vqx_vq_perplexity(const float* counts, int32_t K, int64_t n_rows, float* out, vqx_stream_t stream) {
  if (!counts || !out || K < 1 || n_rows < 1) { set_error("vqx_vq_perplexity: bad arguments"); return -1; }
  hipLaunchKernelGGL(vq_perplexity_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, counts, K, 1.0f / (float)n_rows, out);
  return launch_status("vqx_vq_perplexity");
}

extern "C" int vqx_vq_plain_bwd(const float* z, const float* z_norm, const float* z_len, const float* zq,
                                const void* dzq, const int32_t* src_t, int32_t T, int64_t n_rows, int32_t D,
                                int32_t normalize, float beta, float scale, void* dz, int32_t dtype, const float* bsum,
                                const float* bcnt, const float* emb, const float* e_len, int32_t K, float* dE,
                                vqx_stream_t stream) {
  if (D != 128) { set_error("vqx_vq_plain_bwd: z_dim must be 128"); return -1; }
  if (!z_norm || !zq || !dz || !bsum || !bcnt || !emb || !dE || T < 1 || n_rows < 1 || K < 1 ||
      (normalize && (!z || !z_len || !e_len))) {
    set_error("vqx_vq_plain_bwd: bad arguments");
    return -1;
  }
  const int kb = (K + 3) / 4;
  const int64_t zb = (n_rows + 3) / 4;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == VQX_BF16)
    hipLaunchKernelGGL(vq_plain_bwd_kernel<bf16_t>, dim3((unsigned)(kb + zb)), dim3(256), 0, s, z, z_norm, z_len, zq,
                       (const bf16_t*)dzq, src_t, T, n_rows, normalize, beta, scale, (bf16_t*)dz, bsum, bcnt, emb, e_len,
                       K, dE);
  else
    hipLaunchKernelGGL(vq_plain_bwd_kernel<float>, dim3((unsigned)(kb + zb)), dim3(256), 0, s, z, z_norm, z_len, zq,
                       (const float*)dzq, src_t, T, n_rows, normalize, beta, scale, (float*)dz, bsum, bcnt, emb, e_len,
                       K, dE);
  return launch_status("vqx_vq_plain_bwd");
}
