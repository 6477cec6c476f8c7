// EMA vector quantizer kernels (layers_vq.py:166-334) for gfx950.
//
// vq_forward: one launch does distance -> argmin -> gather -> commitment
// partial sums, reading z in its frame-major layout (no transpose copy,
// layers_vq.py:274-276) and never materialising the (N, K) distance matrix
// (layers_vq.py:285-289); the EMA statistics follow as a dense per-chunk
// reduction (vq_stats_kernel + vq_stats_reduce_kernel).
//
// Geometry: see vq_forward_kernel.  The codebook streams through LDS in
// 64-code steps (XOR-swizzled 16-B chunks so the ds_read_b128 B-fragment
// reads are conflict-free).  Dot products are exact f32 (fmaf chains), the distance
// is formed in the reference's order (||z||^2 + ||e||^2) - 2 z.e, and the
// argmin keeps the first minimum (strict '<' in ascending code order, then
// a lowest-index tie-break across lanes), matching torch.argmin.
#include "vqx_common.h"

#include <cstring>

namespace vqx {

// Code widths D (= z_dim) the kernels are built for: 64, 128 (the BASELINE
// configs) and 256; every vqx_vq_* entry point refuses any other.
inline bool vq_d_ok(int D) { return D == 64 || D == 128 || D == 256; }
// Workgroup geometry of vq_forward_kernel: VQ_FG groups of 16 frames x VQ_CS
// code splits = 8 waves.  A wave keeps its 16 frames' z (16 x D f32) in
// registers as the A operand of v_mfma_f32_16x16x4_f32 and, per step, scores
// them against VQ_SUB codes (one accumulator chain per 16 codes; the 40-cycle
// dependent-MFMA latency is covered by the other waves of the SIMD).  The
// VQ_CS waves of a frame group take disjoint code ranges of the
// step; their (distance, index) minima merge through LDS at the end.  512
// workgroups of 8 waves at 32 KiB LDS and <= 128 VGPRs: two workgroups per
// CU, four waves per SIMD, so one wave's barrier / LDS / epilogue stalls run under another's
// MFMAs (the round-1 kernel had one wave per SIMD).
constexpr int VQ_FG = 2;
constexpr int VQ_CS = 4;
constexpr int VQ_SUB = 16;
constexpr int VQ_STEP = VQ_CS * VQ_SUB;            // 64 codes per LDS step
constexpr int VQ_THREADS = 64 * VQ_FG * VQ_CS;     // 512
constexpr int VQ_FRAMES = 16 * VQ_FG;              // 32 frames per workgroup
template <int D>
constexpr int vq_step_bytes() { return VQ_STEP * D * 4; }  // 32 KiB at D = 128
template <int D>
constexpr int vq_stage() { return vq_step_bytes<D>() / 16 / VQ_THREADS; }  // 16-B chunks staged per thread per step

// EMA statistics (vq_stats_kernel): frames per chunk and the per-code sum
// slabs [chunks][K][D] + counts [chunks][K] that vq_stats_reduce_kernel sums
// in chunk order.
#ifndef VQX_VQ_STATS_DSL_MAX  // widest dim slice (lab builds narrow it: more workgroups per chunk)
#define VQX_VQ_STATS_DSL_MAX 32
#endif
__host__ __device__ constexpr int vq_stats_dsl(int K) {  // dims per LDS slice: K * (dsl + 1) * 4 B + ~10 KiB <= 64 KiB
  int d = VQX_VQ_STATS_DSL_MAX;  // <= 32: a thread holds VQ_CHUNK * dsl / 1024 sorted rows in registers
  while (d > 4 && K * (d + 1) > 13824) d >>= 1;
  return d;
}
inline int vq_stats_chunks(int64_t N, int K) {
  (void)K;
  return (int)((N + 511) / 512);  // VQ_CHUNK frames per chunk
}
inline int64_t vq_partials_floats(int64_t N) { return (N + VQ_FRAMES - 1) / VQ_FRAMES; }
inline int64_t vq_workspace_floats(int64_t N, int K, int D, bool stats) {
  int64_t f = (vq_partials_floats(N) + 63) & ~(int64_t)63;
  if (stats) f += (int64_t)vq_stats_chunks(N, K) * K * (D + 1);
  return f;
}

// D = 256: a 128-KiB double-buffered step leaves one workgroup per CU
template <int D>
__global__ __launch_bounds__(VQ_THREADS, D == 256 ? 2 : 4) void vq_forward_kernel(const float* __restrict__ z, int64_t N,
                                                                   const float* __restrict__ E, int K,
                                                                   int64_t* __restrict__ idx_out,
                                                                   float* __restrict__ zq, void* __restrict__ zq_c,
                                                                   int zq_dt, float* __restrict__ partials) {
  // two code steps in LDS (double buffer) + their ||e||^2: one barrier per step,
  // the next step's LDS writes issued beside this step's MFMAs.  64.5 KiB at
  // D = 128: two workgroups per CU.
  constexpr int VQ_STEP_BYTES = vq_step_bytes<D>(), VQ_STAGE = vq_stage<D>(), KB = D / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * VQ_STEP_BYTES];
  __shared__ float eeL[2][VQ_STEP];
  __shared__ float red[16];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fg = w % VQ_FG, cs = w / VQ_FG;
  const int q = lane >> 4, j16 = lane & 15;
  const int64_t my_row = (int64_t)blockIdx.x * VQ_FRAMES + fg * 16 + j16;  // A-operand row of this lane
  const bool row_ok = my_row < N;

  const int nsteps = (K + VQ_STEP - 1) / VQ_STEP;
  // Staging: thread t holds VQ_STAGE consecutive 16-B chunks (D / 2 bytes) of
  // code t >> 3 of the step, loaded through one buffer descriptor over E (codes
  // >= K read as zeros, no branches) one step ahead of its LDS write.  The 8
  // threads of a code also form its ||e||^2 (the D/8 fmaf of each thread, then
  // two quad-DPP and one half-row-mirror adds) into eeL, so the score loop
  // needs one LDS read per code block.
  static_assert(VQ_STAGE * 8 * 16 == D * 4 && VQ_STEP * 8 == VQ_THREADS, "staging layout");
  const __amdgpu_buffer_rsrc_t rsE =
      __builtin_amdgcn_make_buffer_rsrc((void*)E, (short)0, (int)((int64_t)K * D * 4), 0x00020000);
  const int s_code = tid >> 3, s_part = tid & 7;
  const unsigned s_off = (unsigned)(s_code * D * 4 + s_part * 16 * VQ_STAGE);
  f32x4_t stage[VQ_STAGE];
  auto load_step = [&](int st) {
    typedef float f4v __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int j = 0; j < VQ_STAGE; ++j) {
      const f4v v = __builtin_amdgcn_raw_buffer_load_b128(rsE, (int)(s_off + 16 * j), st * VQ_STEP_BYTES, 0);
      stage[j] = f32x4_t{v[0], v[1], v[2], v[3]};
    }
  };
  auto lds_at = [&](int buf, int code, int ch) {
    return smem + buf * VQ_STEP_BYTES + code * (D * 4) + 16 * (ch ^ (code & 15));
  };
  // the staged step into buffer buf, its codes' squared norms into eeL[buf]
  auto write_step = [&](int buf) {
    float e2 = 0.f;
#pragma unroll
    for (int j = 0; j < VQ_STAGE; ++j) {
      *(f32x4_t*)lds_at(buf, s_code, VQ_STAGE * s_part + j) = stage[j];
      e2 = fmaf(stage[j][0], stage[j][0], e2);
      e2 = fmaf(stage[j][1], stage[j][1], e2);
      e2 = fmaf(stage[j][2], stage[j][2], e2);
      e2 = fmaf(stage[j][3], stage[j][3], e2);
    }
    e2 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, e2), 0xB1, 0xF, 0xF, false));
    e2 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, e2), 0x4E, 0xF, 0xF, false));
    e2 += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, e2), 0x141, 0xF, 0xF, false));
    if (s_part == 0) eeL[buf][s_code] = e2;
  };

  load_step(0);  // the first codebook step and z travel together

  // z fragments: zf[kb] = z[my_row][16kb + 4q .. +3] (rows >= N read as zeros
  // through a descriptor that starts at this workgroup's first frame)
  f32x4_t zf[KB];
  float zz = 0.f;
  const int64_t wg_row0 = (int64_t)blockIdx.x * VQ_FRAMES;
  int64_t z_rec = (N - wg_row0) * D * 4;
  if (z_rec > VQ_FRAMES * D * 4) z_rec = VQ_FRAMES * D * 4;
  const __amdgpu_buffer_rsrc_t rsZ =
      __builtin_amdgcn_make_buffer_rsrc((void*)(z + wg_row0 * D), (short)0, (int)z_rec, 0x00020000);
  const unsigned z_off = (unsigned)((fg * 16 + j16) * (D * 4) + 16 * q);
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v u = __builtin_amdgcn_raw_buffer_load_b128(rsZ, (int)(z_off + 64 * kb), 0, 0);
    const f32x4_t v = {u[0], u[1], u[2], u[3]};
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

  write_step(0);
  if (nsteps > 1) load_step(1);
  __syncthreads();
  const int cbase = cs * VQ_SUB;  // this wave's codes inside a step
  for (int st = 0; st < nsteps; ++st) {
    const int cur = st & 1;
    // step st+1 into the other buffer (its step st-1 readers passed the last
    // barrier); step st+2's loads go out behind it
    if (st + 1 < nsteps) {
      write_step(cur ^ 1);
      if (st + 2 < nsteps) load_step(st + 2);
    }
    constexpr int NB = VQ_SUB / 16;
    // two independent accumulator chains per code block (even / odd 16-dim
    // blocks, added at the end): the 40-cycle dependent-MFMA latency hides
    // under the other chain's 32-cycle issue within the wave
    float eb[NB];
    f32x4_t acc[NB], acc2[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      eb[b] = eeL[cur][cbase + 16 * b + j16];
      acc[b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      acc2[b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int kb = 0; kb < KB; kb += 2) {
      f32x4_t bf[NB], bg[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        bf[b] = *(const f32x4_t*)lds_at(cur, cbase + 16 * b + j16, 4 * kb + q);
        bg[b] = *(const f32x4_t*)lds_at(cur, cbase + 16 * b + j16, 4 * kb + 4 + q);
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(zf[kb][m], bf[b][m], acc[b], 0, 0, 0);
          acc2[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(zf[kb + 1][m], bg[b][m], acc2[b], 0, 0, 0);
        }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] += acc2[b];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int code = st * VQ_STEP + cbase + 16 * b + j16;
      if (code < K) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // codes ascend within a lane, so strict '<' keeps the first minimum
          const float d = __fsub_rn(__fadd_rn(zz_r[r], eb[b]), __fmul_rn(2.f, acc[b][r]));
          if (d < best_d[r]) { best_d[r] = d; best_i[r] = code; }
        }
      }
    }
    __syncthreads();  // step st+1 is in LDS; step st's buffer may be rewritten
  }

  // argmin across the 16 code lanes of each row (lowest index on ties)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      const float od = __shfl_xor(best_d[r], o, 64);
      const int oi = __shfl_xor(best_i[r], o, 64);
      if (od < best_d[r] || (od == best_d[r] && oi < best_i[r])) { best_d[r] = od; best_i[r] = oi; }
    }
  }
  // ... and across the code splits: (distance, index) minima through LDS, merged
  // in ascending split order with the same comparison = torch.argmin's first minimum
  // (the loop's last barrier: no wave reads codes any more)
  float* md = (float*)smem;                       // [VQ_FG][VQ_CS][16]
  int* mi = (int*)(smem + VQ_FG * VQ_CS * 16 * 4);
  if (j16 == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      md[(fg * VQ_CS + cs) * 16 + 4 * q + r] = best_d[r];
      mi[(fg * VQ_CS + cs) * 16 + 4 * q + r] = best_i[r];
    }
  }
  __syncthreads();
  float sq = 0.f;
  if (cs == 0) {  // the frame group's epilogue (every split wave holds the same z)
    float bd = md[fg * VQ_CS * 16 + j16];
    int bi = mi[fg * VQ_CS * 16 + j16];
#pragma unroll
    for (int c = 1; c < VQ_CS; ++c) {
      const float od = md[(fg * VQ_CS + c) * 16 + j16];
      const int oi = mi[(fg * VQ_CS + c) * 16 + j16];
      if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; }
    }
    // NaN rows (every comparison false) keep a well-defined index
    const int my_idx = (bi >= K || bi < 0) ? 0 : bi;
    if (row_ok) {
      if (q == 0) idx_out[my_row] = my_idx;
      // the code row's 8 loads all in flight before the first store (a
      // load-store pair per 16 dims paid one memory latency each)
      f32x4_t ev[KB];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) ev[kb] = *(const f32x4_t*)(E + (int64_t)my_idx * D + 16 * kb + 4 * q);
      if (zq) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) *(f32x4_t*)(zq + my_row * D + 16 * kb + 4 * q) = ev[kb];
      }
      if (zq_c && zq_dt == VQX_BF16) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
          uint2 pk;
          pk.x = pack_bf16x2(ev[kb][0], ev[kb][1]);
          pk.y = pack_bf16x2(ev[kb][2], ev[kb][3]);
          *(uint2*)((bf16_t*)zq_c + my_row * D + 16 * kb + 4 * q) = pk;
        }
      } else if (zq_c) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) *(f32x4_t*)((float*)zq_c + my_row * D + 16 * kb + 4 * q) = ev[kb];
      }
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const float df = __fsub_rn(ev[kb][m], zf[kb][m]);
          sq = fmaf(df, df, sq);
        }
    }
  }
  const float tot = block_sum(sq, red);
  if (tid == 0) partials[blockIdx.x] = tot;
}

// EMA statistics (update_emb, layers_vq.py:207-211: onehot(idx) @ z and the
// code counts) as a dense per-chunk reduction, deterministic and free of
// atomics: workgroup (chunk c of <= VQ_CHUNK frames, dim slice y of DSL
// dims) bitonic-sorts its frames by (code, frame) in LDS; thread (g, r) then
// sums 4 dims of the r-th range of sorted frames, writing every run that lies
// inside its range straight into the LDS table [K][DSL] and leaving the two
// runs cut by range edges as partials, which the thread holding each run's
// first frame completes in ascending range order.  The table becomes the
// chunk's slab row; vq_stats_reduce_kernel sums the slabs in chunk order.
// (LDS float atomics measured ~11 us of an 18 us kernel: ~one lane per clock.)
constexpr int VQ_CHUNK = 512;

template <int DSL>
__global__ __launch_bounds__(256) void vq_stats_kernel(const float* __restrict__ z, int64_t N, int D,
                                                       const int64_t* __restrict__ idx, int K, int64_t frames_per_chunk,
                                                       float* __restrict__ slab, float* __restrict__ cnt_slab) {
  constexpr int G = DSL / 4;             // 4-dim groups per slice
  constexpr int R = 256 / G;             // ranges of sorted frames
  constexpr int LEN = VQ_CHUNK / R;      // sorted frames per range
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* acc = lds;                                  // [K][DSL]
  int* keys = (int*)(acc + K * DSL);                 // [VQ_CHUNK] code << 9 | frame (sorted)
  int* runk = keys + VQ_CHUNK;                       // [R][2] head / tail run code (-1: none)
  int* cnt = runk + 2 * R;                           // [K] (slice 0)
  f32x4_t* part = (f32x4_t*)(cnt + ((K + 3) & ~3));  // [R][2][G] head / tail partial sums
  const int tid = threadIdx.x;
  const int c = blockIdx.x, d0 = blockIdx.y * DSL;
  const bool counts = blockIdx.y == 0;
  const int64_t n0 = (int64_t)c * frames_per_chunk;
  const int nf = (int)((n0 + frames_per_chunk < N ? n0 + frames_per_chunk : N) - n0);
  for (int i = tid; i < K * DSL; i += 256) acc[i] = 0.f;
  if (counts)
    for (int i = tid; i < K; i += 256) cnt[i] = 0;
  {
    // both index loads in flight at once (clamped to the chunk's last frame,
    // the frames past it marked invalid after the load)
    static_assert(VQ_CHUNK == 2 * 256, "two keys per thread");
    int64_t iv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) iv[u] = idx[n0 + min(tid + 256 * u, nf - 1)];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = tid + 256 * u;
      int code = i < nf ? (int)iv[u] : K;
      if (code < 0 || code > K) code = K;  // out-of-range codes sort last and are dropped
      keys[i] = code < K ? (code << 9) | i : 0x7fffffff;
    }
  }
  __syncthreads();
  if (counts)
    for (int i = tid; i < nf; i += 256) {
      const int k = keys[i];
      if (k != 0x7fffffff) atomicAdd(&cnt[k >> 9], 1);  // integer counts: exact in any order
    }
  __syncthreads();  // the count loop reads keys[] that the sort's first pass swaps
  // bitonic sort, ascending (VQ_CHUNK = 2 elements per thread per step)
  for (int k = 2; k <= VQ_CHUNK; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int i = 2 * tid - (tid & (j - 1));
      const int a = keys[i], b = keys[i + j];
      const bool up = (i & k) == 0;
      if ((a > b) == up) { keys[i] = b; keys[i + j] = a; }
      __syncthreads();
    }
  }
  // segmented sums over range r, 4 dims (group g)
  const int g = tid % G, r = tid / G, dd = d0 + 4 * g;
  const int p0 = r * LEN;
  f32x4_t rows[LEN];
  int rc[LEN];
  // every row load of the thread in flight at once (invalid keys read frame 0
  // of the chunk and are zeroed after the load)
#pragma unroll
  for (int u = 0; u < LEN; ++u) {
    const int key = keys[p0 + u];
    rc[u] = key == 0x7fffffff ? -1 : key >> 9;
    rows[u] = *(const f32x4_t*)(z + (n0 + (rc[u] < 0 ? 0 : (key & 511))) * D + dd);
  }
#pragma unroll
  for (int u = 0; u < LEN; ++u)
    if (rc[u] < 0) rows[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  f32x4_t run = rows[0];
  int cur = rc[0];
  bool head = true;
#pragma unroll
  for (int u = 1; u <= LEN; ++u) {
    const int nc = u < LEN ? rc[u] : -2;
    if (nc != cur) {
      if (head) {  // first run of the range: may have started in an earlier range
        part[(r * 2 + 0) * G + g] = run;
        if (g == 0) runk[2 * r] = cur;
        head = false;
      } else if (u == LEN) {  // last run: may continue into the next range
        part[(r * 2 + 1) * G + g] = run;
        if (g == 0) runk[2 * r + 1] = cur;
      } else if (cur >= 0) {  // a run wholly inside the range: exclusive
        *(f32x4_t*)&acc[cur * DSL + 4 * g] = run;
      }
      if (u < LEN) { run = rows[u]; cur = nc; }
    } else {
      run += rows[u];
    }
  }
  if (head == false && g == 0 && rc[LEN - 1] == runk[2 * r]) {
    // the range is one run: the head partial also serves as its tail
    runk[2 * r + 1] = -1;
  }
  __syncthreads();
  // complete the runs cut by range edges: the range holding a run's first frame
  // adds the continuations in ascending range order
  auto finish = [&](int code, int rr, f32x4_t sum) {
    for (int q = rr + 1; q < R; ++q) {
      if (runk[2 * q] != code) break;
      sum += part[(q * 2 + 0) * G + g];
      if (runk[2 * q + 1] != -1) break;  // the run ends inside range q
    }
    *(f32x4_t*)&acc[code * DSL + 4 * g] = sum;
  };
  {
    const int kh = runk[2 * r];
    // the head run starts here unless the previous range ends with the same code
    const int prev_tail = r > 0 ? (runk[2 * (r - 1) + 1] != -1 ? runk[2 * (r - 1) + 1] : runk[2 * (r - 1)]) : -3;
    if (kh >= 0 && kh != prev_tail) {
      if (runk[2 * r + 1] == -1) finish(kh, r, part[(r * 2 + 0) * G + g]);          // single run: may continue
      else *(f32x4_t*)&acc[kh * DSL + 4 * g] = part[(r * 2 + 0) * G + g];          // ends inside the range
    }
    const int kt = runk[2 * r + 1];
    if (kt >= 0) finish(kt, r, part[(r * 2 + 1) * G + g]);
  }
  __syncthreads();
  float* out = slab + (int64_t)c * K * D + d0;
  for (int i = tid; i < K * G; i += 256) {
    const int k = i / G, q = i % G;
    *(f32x4_t*)(out + (int64_t)k * D + 4 * q) = *(const f32x4_t*)&acc[k * DSL + 4 * q];
  }
  if (counts)
    for (int i = tid; i < K; i += 256) cnt_slab[(int64_t)c * K + i] = (float)cnt[i];
}

// bsum[i] += sum_c slab[c][i], bcnt[k] += sum_c cnt_slab[c][k], summed in
// chunk order: 64 float4 columns per workgroup, 4 threads per column each
// loading a quarter of the chunks (independent loads), combined in order.
__global__ __launch_bounds__(256) void vq_stats_reduce_kernel(const float* __restrict__ slab,
                                                              const float* __restrict__ cnt_slab, int chunks, int K,
                                                              int D, float* __restrict__ bsum,
                                                              float* __restrict__ bcnt) {
  __shared__ f32x4_t red[4][64];
  const int64_t total = (int64_t)K * D;
  const int col = threadIdx.x & 63, qg = threadIdx.x >> 6;
  const int64_t i4 = ((int64_t)blockIdx.x * 64 + col) * 4;
  const int per = (chunks + 3) / 4, c0 = qg * per, c1 = min(chunks, c0 + per);
  f32x4_t s = {0.f, 0.f, 0.f, 0.f};
  if (i4 < total) {
    int c = c0;
    for (; c + 8 <= c1; c += 8) {
      f32x4_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *(const f32x4_t*)(slab + (int64_t)(c + u) * total + i4);
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; c < c1; ++c) s += *(const f32x4_t*)(slab + (int64_t)c * total + i4);
  }
  red[qg][col] = s;
  __syncthreads();
  if (qg == 0 && i4 < total) {
    const f32x4_t t = ((red[0][col] + red[1][col]) + red[2][col]) + red[3][col];
    *(f32x4_t*)(bsum + i4) = *(f32x4_t*)(bsum + i4) + t;
  }
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (bcnt && k < K) {
    float t = 0.f;
    int c = 0;
    for (; c + 8 <= chunks; c += 8) {  // independent loads in flight (the sum order stays 0, 1, 2, ...)
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = cnt_slab[(int64_t)(c + u) * K + k];
#pragma unroll
      for (int u = 0; u < 8; ++u) t += v[u];
    }
    for (; c < chunks; ++c) t += cnt_slab[(int64_t)c * K + k];
    bcnt[k] += t;
  }
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
// EMA update in one launch: the K*D elementwise update over many workgroups
// (one exact division per element; a single workgroup took ~48 us), each
// storing its squared-difference partial; the last workgroup to finish
// (arrive_last, counter after the partials) then runs the per-code terms, the
// emb_elem update and the diagnostics, summing the partials in a fixed order
// (deterministic).  Round 6: the per-code pass was a second, one-workgroup
// launch (1024 threads; ~5 us).
constexpr int kEmaElems = 1024;  // elements per workgroup of vq_ema_kernel

// row indices passed by value (vqx_gather_rows_host): kernel arguments, no copy on the stream
constexpr int kGatherArgRows = 512;
struct GatherIdx {
  int32_t idx[kGatherArgRows];
};

// The step's closing work in the last workgroup (vqx_vq_ema_update_close):
// up to two fixed-order sums (the log-loss total and the commitment sum that
// sum_partials2_kernel computed) and the mailbox publish of the statistics
// (mailbox_publish_kernel, vqx_runtime.hip).
struct CloseArgs {
  const float* parts[2];
  int n[2];
  float scale[2];
  float* out[2];
  const float* pub_src;
  int pub_n;
  float* pub_copy;
  float* pub_box;     // the slot's values (mapped host memory)
  uint32_t* pub_seqp;  // the slot's sequence number
  uint32_t pub_seq;
};

// The per-code pass and the closing work in one 256-thread workgroup.  Every
// sum is the one the 1024-thread launches it replaces formed (block_sum_nv:
// four virtual threads per thread), so the diagnostics and the loss sums keep
// their bits.
constexpr int kEmaNV = 4;  // 1024 / 256
__device__ __forceinline__ void ema_final_block(float* emb_elem, const float* bcnt, int K, int D, float mu,
                                                float one_minus_mu, float thr, const float* __restrict__ part,
                                                int nparts, float* __restrict__ diag, float* clear_cnt,
                                                const CloseArgs& C) {
  __shared__ float red[3][16];
  constexpr int NV = kEmaNV;
  const int nt = blockDim.x, vt = NV * nt;
  if (C.parts[0] || C.parts[1]) {  // sum_partials2_kernel: thread-strided sums, then the block sum
    float v[2][NV], o[2];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int t = threadIdx.x + j * nt;
      v[0][j] = v[1][j] = 0.f;
      for (int i = t; i < C.n[0]; i += vt) v[0][j] += C.parts[0][i];
      for (int i = t; i < C.n[1]; i += vt) v[1][j] += C.parts[1][i];
    }
    block_sum_nv<2, NV>(v, red, o);
    if (threadIdx.x == 0) {
      if (C.out[0]) C.out[0][0] = o[0] * C.scale[0];
      if (C.out[1]) C.out[1][0] = o[1] * C.scale[1];
    }
    __syncthreads();  // red is rewritten
  }
  float a[2][NV], ao[2];  // sum of squared codebook moves, total count
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int t = threadIdx.x + j * nt;
    a[0][j] = a[1][j] = 0.f;
    for (int b = t; b < nparts; b += vt) a[0][j] += ld_agent(part + b);
    for (int k = t; k < K; k += vt) a[1][j] += bcnt[k];
  }
  block_sum_nv<2, NV>(a, red, ao);
  const float dsq = ao[0], total = ao[1];
  float e[3][NV], eo[3];  // entropy term, codes used this step, codes in use after the update
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int t = threadIdx.x + j * nt;
    e[0][j] = e[1][j] = e[2][j] = 0.f;
    for (int k = t; k < K; k += vt) {
      const float c = bcnt[k];
      const float p = c / total;
      e[0][j] += p * logf(p + 1e-8f);
      e[1][j] += (c >= thr) ? 1.f : 0.f;
      const float el = __fadd_rn(__fmul_rn(mu, emb_elem[k]), __fmul_rn(one_minus_mu, c));
      e[2][j] += (el >= thr) ? 1.f : 0.f;
    }
  }
  __syncthreads();  // red is rewritten
  block_sum_nv<3, NV>(e, red, eo);
  for (int k = threadIdx.x; k < K; k += nt) {
    emb_elem[k] = __fadd_rn(__fmul_rn(mu, emb_elem[k]), __fmul_rn(one_minus_mu, bcnt[k]));
    if (clear_cnt) clear_cnt[k] = 0.f;  // every workgroup's reads of bcnt[k] are done (all arrived)
  }
  if (threadIdx.x == 0) {
    diag[0] = expf(-eo[0]);
    diag[1] = eo[1];
    diag[2] = eo[2];
    diag[3] = sqrtf(dsq) / sqrtf((float)K * (float)D);
  }
  if (!C.pub_seqp) return;
  __syncthreads();  // thread 0's statistics (diag, sums) are in pub_src
  const int t = threadIdx.x;
  if (t < C.pub_n) {
    const float v = C.pub_src[t];
    if (C.pub_copy) C.pub_copy[t] = v;
    __hip_atomic_store(C.pub_box + t, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the values before the number
  __syncthreads();
  if (t == 0) __hip_atomic_store(C.pub_seqp, C.pub_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// emb_elem is read by every workgroup and rewritten by the last one, after
// all have arrived (so not __restrict__)
__global__ __launch_bounds__(256) void vq_ema_kernel(float* __restrict__ emb_sum, float* emb_elem,
                                                     float* __restrict__ E, const float* __restrict__ bsum,
                                                     const float* bcnt, const float* __restrict__ rand_rows, int K,
                                                     int D, float mu, float one_minus_mu, float thr,
                                                     float* __restrict__ part, float* clear_sum,
                                                     float* __restrict__ diag, float* clear_cnt, CloseArgs C,
                                                     const float* __restrict__ rsrc, int rld, GatherIdx R) {
  __shared__ float red[16];
  const int i0 = blockIdx.x * kEmaElems;
  const int n = K * D;
  float dsq = 0.f;
  // the thread's elements' loads all issued first (clamped indices), then the
  // math in element order: a load-use loop paid one memory latency per element
  constexpr int U = kEmaElems / 256;
  static_assert(U * 256 == kEmaElems, "elements per thread");
  float es[U], bs[U], ee[U], bc[U], rr[U], eo[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = min(i0 + (int)threadIdx.x + 256 * u, n - 1), k = i / D;
    es[u] = emb_sum[i];
    bs[u] = bsum[i];
    ee[u] = emb_elem[k];
    bc[u] = bcnt[k];
    if (rsrc) {  // the dead-code row straight from z (vqx_step_close.rows_src; negative: a zero row)
      const int r = R.idx[k];
      rr[u] = r >= 0 ? rsrc[(int64_t)r * rld + (i - k * D)] : 0.f;
    } else {
      rr[u] = rand_rows[i];
    }
    eo[u] = E[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = i0 + (int)threadIdx.x + 256 * u;
    if (i >= n) break;
    const float s = __fadd_rn(__fmul_rn(mu, es[u]), __fmul_rn(one_minus_mu, bs[u]));
    const float el = __fadd_rn(__fmul_rn(mu, ee[u]), __fmul_rn(one_minus_mu, bc[u]));
    emb_sum[i] = s;
    if (clear_sum) clear_sum[i] = 0.f;  // consumed: zero for the next step's accumulation
    const float uu = (el >= thr) ? 1.f : 0.f;
    // usage*(sum/elem) + (1-usage)*rand, evaluated like the reference
    const float newe = __fadd_rn(__fmul_rn(uu, __fdiv_rn(s, el)), __fmul_rn(1.f - uu, rr[u]));
    const float diff = __fsub_rn(newe, eo[u]);
    dsq = fmaf(diff, diff, dsq);
    E[i] = newe;
  }
  dsq = block_sum(dsq, red);
  if (threadIdx.x == 0) st_agent(part + blockIdx.x, dsq);
  if (!arrive_last((unsigned*)(part + gridDim.x), gridDim.x)) return;
  ema_final_block(emb_elem, bcnt, K, D, mu, one_minus_mu, thr, part, gridDim.x, diag, clear_cnt, C);
}

__global__ void gather_rows_kernel(const float* __restrict__ src, int ld, const int64_t* __restrict__ rows,
                                   int n_out, int D, float* __restrict__ out) {
  const int i = blockIdx.x;
  if (i >= n_out) return;
  const int64_t r = rows[i];
  for (int d = threadIdx.x; d < D; d += blockDim.x) out[(int64_t)i * D + d] = (r >= 0) ? src[r * ld + d] : 0.f;
}

__global__ void gather_rows_arg_kernel(const float* __restrict__ src, int ld, GatherIdx R, int n_out, int D,
                                       float* __restrict__ out) {
  const int i = blockIdx.x;
  if (i >= n_out) return;
  const int64_t r = R.idx[i];
  for (int d = threadIdx.x; d < D; d += blockDim.x) out[(int64_t)i * D + d] = (r >= 0) ? src[r * ld + d] : 0.f;
}

template <typename T>
__global__ void commit_bwd_kernel(const float* __restrict__ z, const float* __restrict__ zq, int64_t n, float scale,
                                  T* __restrict__ dz) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    Elem<T>::st(dz, i, scale * __fsub_rn(z[i], zq[i]));
}

// commit_bwd with the column sums of the stored dz: block p = row part p,
// thread = (4-column chunk, row group); rows of a group four at a time (their
// loads in flight together), the groups' sums added in order through LDS.
template <typename T>
__global__ __launch_bounds__(256) void commit_bwd_cs_kernel(const float* __restrict__ z, const float* __restrict__ zq,
                                                            int64_t n_rows, int D, float scale, T* __restrict__ dz,
                                                            float* __restrict__ part) {
  const int cpr = D / 4, R = 256 / cpr;
  const int ch = threadIdx.x % cpr, rg = threadIdx.x / cpr;
  const int p = blockIdx.x;
  const int64_t r0 = n_rows * p / VQX_COMMIT_PARTS, r1 = n_rows * (p + 1) / VQX_COMMIT_PARTS;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  auto one = [&](const f32x4_t& a, const f32x4_t& b, int64_t r) {
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = scale * __fsub_rn(a[k], b[k]);
    if constexpr (sizeof(T) == 2) {
      uint2 pk;
      pk.x = pack_bf16x2(v[0], v[1]);
      pk.y = pack_bf16x2(v[2], v[3]);
      *(uint2*)(dz + r * D + 4 * ch) = pk;
      // the column sums are of the values stored
      v[0] = __uint_as_float(pk.x << 16); v[1] = __uint_as_float(pk.x & 0xffff0000u);
      v[2] = __uint_as_float(pk.y << 16); v[3] = __uint_as_float(pk.y & 0xffff0000u);
    } else {
      *(f32x4_t*)(dz + r * D + 4 * ch) = f32x4_t{v[0], v[1], v[2], v[3]};
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] += v[k];
  };
  if (rg < R) {
    int64_t r = r0 + rg;
    for (; r + 3 * R < r1; r += 4 * R) {
      f32x4_t a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = *(const f32x4_t*)(z + (r + u * R) * D + 4 * ch);
        b[u] = *(const f32x4_t*)(zq + (r + u * R) * D + 4 * ch);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) one(a[u], b[u], r + u * R);
    }
    for (; r < r1; r += R) one(*(const f32x4_t*)(z + r * D + 4 * ch), *(const f32x4_t*)(zq + r * D + 4 * ch), r);
  }
  __shared__ float lds[256 * 4];
#pragma unroll
  for (int k = 0; k < 4; ++k) lds[threadIdx.x * 4 + k] = s[k];
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    const int cc = c >> 2, k = c & 3;
    float t = 0.f;
    for (int q = 0; q < R; ++q) t += lds[(q * cpr + cc) * 4 + k];
    part[(int64_t)p * D + c] = t;
  }
}

}  // namespace vqx

using namespace vqx;

extern "C" int vqx_vq_workspace(int64_t n_rows, int32_t K, int32_t D, int32_t with_stats, int64_t* floats) {
  if (n_rows <= 0 || K <= 0 || !floats || !vq_d_ok(D)) { set_error("vqx_vq_workspace: bad arguments"); return -1; }
  *floats = vq_workspace_floats(n_rows, K, D, with_stats != 0);
  return 0;
}

template <int DSL>
static void launch_vq_stats(const float* z, int64_t N, int D, const int64_t* idx, int K, float* ws, float* bsum,
                            float* bcnt, hipStream_t s) {
  const int chunks = vq_stats_chunks(N, K);
  const int64_t fpc = VQ_CHUNK;
  float* slab = ws + ((vq_partials_floats(N) + 63) & ~(int64_t)63);
  float* cnt_slab = slab + (int64_t)chunks * K * D;
  constexpr int R = 256 / (DSL / 4);
  const size_t lds = (size_t)K * DSL * 4 + VQ_CHUNK * 4 + 2 * R * 4 + (size_t)((K + 3) & ~3) * 4 + 2 * R * (DSL / 4) * 16;
  hipLaunchKernelGGL(vq_stats_kernel<DSL>, dim3(chunks, D / DSL), dim3(256), lds, s, z, N, D, idx, K, fpc, slab,
                     cnt_slab);
  const int64_t total4 = (int64_t)K * D / 4;
  unsigned nb = (unsigned)((total4 + 63) / 64);
  if (nb * 256u < (unsigned)K) nb = (unsigned)((K + 255) / 256);
  hipLaunchKernelGGL(vq_stats_reduce_kernel, dim3(nb), dim3(256), 0, s, slab, cnt_slab, chunks, K, D, bsum, bcnt);
}

extern "C" int vqx_vq_forward(const float* z, int64_t n_rows, int32_t D, const float* E, int32_t K, int64_t* idx,
                              float* zq, void* zq_c, int32_t zq_c_dtype, float* sqerr_out, float* partials,
                              float* bsum, float* bcnt, vqx_stream_t stream) {
  if (!vq_d_ok(D)) { set_error("vqx_vq_forward: D must be 64, 128 or 256 (got %d)", D); return -1; }
  if (K <= 0 || K % 16) { set_error("vqx_vq_forward: K=%d must be a positive multiple of 16", K); return -1; }
  if (bsum && K > 2048) { set_error("vqx_vq_forward: EMA statistics need K <= 2048 (got %d)", K); return -1; }
  if (n_rows <= 0 || !z || !E || !idx || !partials) { set_error("vqx_vq_forward: bad arguments"); return -1; }
  if (bcnt && !bsum) { set_error("vqx_vq_forward: bcnt needs bsum"); return -1; }
  if (((uintptr_t)z | (uintptr_t)E) & 15) { set_error("vqx_vq_forward: z/E must be 16-byte aligned"); return -1; }
  hipStream_t s = (hipStream_t)stream;
  const int grid = (int)vq_partials_floats(n_rows);
  auto* kfn = D == 64 ? vq_forward_kernel<64> : D == 128 ? vq_forward_kernel<128> : vq_forward_kernel<256>;
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(VQ_THREADS), 0, s, z, n_rows, E, K, idx, zq, zq_c, zq_c_dtype, partials);
  if (sqerr_out) hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(1024), 0, s, partials, grid, 1.0f, sqerr_out);
  if (bsum) {
    switch (vq_stats_dsl(K)) {
      case 32: launch_vq_stats<32>(z, n_rows, D, idx, K, partials, bsum, bcnt, s); break;
      case 16: launch_vq_stats<16>(z, n_rows, D, idx, K, partials, bsum, bcnt, s); break;
      case 8: launch_vq_stats<8>(z, n_rows, D, idx, K, partials, bsum, bcnt, s); break;
      default: launch_vq_stats<4>(z, n_rows, D, idx, K, partials, bsum, bcnt, s); break;
    }
  }
  return launch_status("vqx_vq_forward");
}

extern "C" int vqx_vq_stats(const float* z, int64_t n_rows, int32_t D, const int64_t* idx, int32_t K,
                            float* partials, float* bsum, float* bcnt, vqx_stream_t stream) {
  if (!vq_d_ok(D)) { set_error("vqx_vq_stats: D must be 64, 128 or 256 (got %d)", D); return -1; }
  if (K <= 0 || K % 16 || K > 2048) { set_error("vqx_vq_stats: K=%d must be a multiple of 16 in [16, 2048]", K); return -1; }
  if (n_rows <= 0 || !z || !idx || !partials || !bsum || !bcnt) { set_error("vqx_vq_stats: bad arguments"); return -1; }
  if ((uintptr_t)z & 15) { set_error("vqx_vq_stats: z must be 16-byte aligned"); return -1; }
  hipStream_t s = (hipStream_t)stream;
  switch (vq_stats_dsl(K)) {
    case 32: launch_vq_stats<32>(z, n_rows, D, idx, K, partials, bsum, bcnt, s); break;
    case 16: launch_vq_stats<16>(z, n_rows, D, idx, K, partials, bsum, bcnt, s); break;
    case 8: launch_vq_stats<8>(z, n_rows, D, idx, K, partials, bsum, bcnt, s); break;
    default: launch_vq_stats<4>(z, n_rows, D, idx, K, partials, bsum, bcnt, s); break;
  }
  return launch_status("vqx_vq_stats");
}

static int ema_update(float* emb_sum, float* emb_elem, float* E, const float* bsum, const float* bcnt,
                      const float* rand_rows, int32_t K, int32_t D, float mu, float threshold, float* diag,
                      float* partials, bool clear, const vqx_step_close* close, vqx_stream_t stream) {
  if (K <= 0 || D <= 0 || !partials || !diag) { set_error("vqx_vq_ema_update: bad K/D, no partials or no diag"); return -1; }
  CloseArgs C{};
  GatherIdx R;
  const float* rsrc = nullptr;
  int rld = 0;
  if (close && close->rows_src) {
    if (close->n_rows != K || K > kGatherArgRows || !close->rows_host || close->rows_ld < D) {
      set_error("vqx_vq_ema_update_close: rows_src needs n_rows == K <= %d host indices and ld >= D", kGatherArgRows);
      return -1;
    }
    for (int i = 0; i < K; ++i) R.idx[i] = close->rows_host[i];
    rsrc = close->rows_src;
    rld = close->rows_ld;
  } else if (!rand_rows) {
    set_error("vqx_vq_ema_update: no rand_rows");
    return -1;
  }
  if (close) {
    for (int i = 0; i < 2; ++i) {
      if (close->parts[i] && (close->n[i] < 0 || !close->out[i])) { set_error("vqx_vq_ema_update_close: sum %d needs n >= 0 and an output", i); return -1; }
      C.parts[i] = close->parts[i];
      C.n[i] = close->parts[i] ? close->n[i] : 0;
      C.scale[i] = close->scale[i];
      C.out[i] = close->parts[i] ? close->out[i] : nullptr;
    }
    if (close->pub_box) {
      const int n = close->pub_n, slots = close->pub_slots, fl = close->pub_floats, slot = close->pub_slot;
      if (!close->pub_src || n < 1 || n > fl || fl > 64 || slot < 0 || slot >= slots) {
        set_error("vqx_vq_ema_update_close: bad mailbox arguments");
        return -1;
      }
      C.pub_src = close->pub_src;
      C.pub_n = n;
      C.pub_copy = close->pub_copy;
      C.pub_seqp = (uint32_t*)close->pub_box + slot;
      C.pub_box = (float*)((uint32_t*)close->pub_box + slots) + (size_t)slot * fl;
      C.pub_seq = close->pub_seq;
    }
  }
  const float omm = (float)(1.0 - (double)mu);  // (1. - mu) in double, as the reference's Python float
  const int nb = (K * D + kEmaElems - 1) / kEmaElems;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(vq_ema_kernel, dim3(nb), dim3(256), 0, s, emb_sum, emb_elem, E, bsum, bcnt, rand_rows, K, D, mu,
                     omm, threshold, partials, clear ? (float*)bsum : nullptr, diag, clear ? (float*)bcnt : nullptr, C,
                     rsrc, rld, R);
  return launch_status("vqx_vq_ema_update");
}

extern "C" int vqx_vq_ema_update(float* emb_sum, float* emb_elem, float* E, const float* bsum, const float* bcnt,
                                 const float* rand_rows, int32_t K, int32_t D, float mu, float threshold, float* diag,
                                 float* partials, vqx_stream_t stream) {
  return ema_update(emb_sum, emb_elem, E, bsum, bcnt, rand_rows, K, D, mu, threshold, diag, partials, false, nullptr,
                    stream);
}

extern "C" int vqx_vq_ema_update_clear(float* emb_sum, float* emb_elem, float* E, float* bsum, float* bcnt,
                                       const float* rand_rows, int32_t K, int32_t D, float mu, float threshold,
                                       float* diag, float* partials, vqx_stream_t stream) {
  if (!bsum || !bcnt) { set_error("vqx_vq_ema_update_clear: null statistics"); return -1; }
  return ema_update(emb_sum, emb_elem, E, bsum, bcnt, rand_rows, K, D, mu, threshold, diag, partials, true, nullptr,
                    stream);
}

extern "C" int vqx_vq_ema_update_close(float* emb_sum, float* emb_elem, float* E, float* bsum, float* bcnt,
                                       const float* rand_rows, int32_t K, int32_t D, float mu, float threshold,
                                       float* diag, float* partials, const vqx_step_close* close,
                                       vqx_stream_t stream) {
  if (!close) { set_error("vqx_vq_ema_update_close: null close arguments"); return -1; }
  return ema_update(emb_sum, emb_elem, E, bsum, bcnt, rand_rows, K, D, mu, threshold, diag, partials, true, close,
                    stream);
}

extern "C" int vqx_gather_rows(const float* src, int32_t ld_src, const int64_t* rows, int32_t n_out, int32_t D,
                               float* out, vqx_stream_t stream) {
  if (n_out <= 0 || D <= 0) { set_error("vqx_gather_rows: bad sizes"); return -1; }
  hipLaunchKernelGGL(gather_rows_kernel, dim3(n_out), dim3(128), 0, (hipStream_t)stream, src, ld_src, rows, n_out, D,
                     out);
  return launch_status("vqx_gather_rows");
}

extern "C" int vqx_gather_rows_host(const float* src, int32_t ld_src, const int32_t* rows, int32_t n_out, int32_t D,
                                    float* out, vqx_stream_t stream) {
  if (n_out <= 0 || D <= 0 || !rows || !src || !out || ld_src < D) {
    set_error("vqx_gather_rows_host: bad arguments");
    return -1;
  }
  for (int i0 = 0; i0 < n_out; i0 += kGatherArgRows) {
    GatherIdx R;
    const int n = std::min(kGatherArgRows, n_out - i0);
    memcpy(R.idx, rows + i0, sizeof(int32_t) * n);
    hipLaunchKernelGGL(gather_rows_arg_kernel, dim3(n), dim3(128), 0, (hipStream_t)stream, src, ld_src, R, n, D,
                       out + (int64_t)i0 * D);
  }
  return launch_status("vqx_gather_rows_host");
}

extern "C" int vqx_vq_commit_bwd_cs(const float* z, const float* zq, int64_t n_rows, int32_t D, float scale, void* dz,
                                    int32_t dtype, float* partials, vqx_stream_t stream) {
  if (!z || !zq || !dz || !partials || n_rows <= 0 || D <= 0 || D % 4 || D > 1024 || 256 % (D / 4) ||
      (((uintptr_t)z | (uintptr_t)zq | (uintptr_t)dz) & 7)) {
    set_error("vqx_vq_commit_bwd_cs: bad arguments (D %% 4 == 0, D / 4 dividing 256, aligned rows)");
    return -1;
  }
  if (dtype == VQX_BF16)
    hipLaunchKernelGGL(commit_bwd_cs_kernel<bf16_t>, dim3(VQX_COMMIT_PARTS), dim3(256), 0, (hipStream_t)stream, z, zq,
                       n_rows, D, scale, (bf16_t*)dz, partials);
  else
    hipLaunchKernelGGL(commit_bwd_cs_kernel<float>, dim3(VQX_COMMIT_PARTS), dim3(256), 0, (hipStream_t)stream, z, zq,
                       n_rows, D, scale, (float*)dz, partials);
  return launch_status("vqx_vq_commit_bwd_cs");
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
// reduction 'frame_mean', target_norm 1.0).  One wave per D-wide row.
// ===================================================================
namespace {

__device__ __forceinline__ float wave_sum64(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// PL = D/64 consecutive floats of a D-wide row per lane (one wave per row)
template <int PL>
struct RowPL {
  float v[PL];
  __device__ __forceinline__ void load(const float* p) {
#pragma unroll
    for (int i = 0; i < PL; ++i) v[i] = p[i];
  }
  __device__ __forceinline__ void store(float* p) const {
#pragma unroll
    for (int i = 0; i < PL; ++i) p[i] = v[i];
  }
  __device__ __forceinline__ float dot(const RowPL& o) const {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PL; ++i) s += v[i] * o.v[i];
    return s;
  }
};

// Blocks [0, ceil(K/4)) renormalise the codebook rows, the rest the frames.
//   codebook (embed_norm, layers_vq.py:28-33, then :99): E *= 1/||E|| in
//     place, embn = (1.0*E)/||E||, e_len = ||E|| (after the in-place step);
//   frames (:97): z_norm = (1.0*z)/||z||, z_len = ||z||, and the per-block
//     sum of (z_norm - z)^2 (normalisation loss, :125-126).
template <int PL>
__global__ __launch_bounds__(256) void vq_normalize_kernel(const float* __restrict__ z, int64_t N, float* __restrict__ E,
                                                           int K, float* __restrict__ zn, float* __restrict__ zlen,
                                                           float* __restrict__ embn, float* __restrict__ elen,
                                                           float* __restrict__ part) {
  constexpr int D = 64 * PL;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kb = (K + 3) / 4;
  __shared__ float red[4];
  if ((int)blockIdx.x < kb) {
    const int k = blockIdx.x * 4 + w;
    if (k >= K) return;
    float* er = E + (int64_t)k * D + PL * lane;
    RowPL<PL> e;
    e.load(er);
    const float n1 = sqrtf(wave_sum64(e.dot(e)));
    const float f = 1.0f / n1;
#pragma unroll
    for (int i = 0; i < PL; ++i) e.v[i] *= f;
    e.store(er);
    const float n2 = sqrtf(wave_sum64(e.dot(e)));
    RowPL<PL> o;
#pragma unroll
    for (int i = 0; i < PL; ++i) o.v[i] = e.v[i] / n2;
    o.store(embn + (int64_t)k * D + PL * lane);
    if (lane == 0) elen[k] = n2;
    return;
  }
  const int64_t n = (int64_t)(blockIdx.x - kb) * 4 + w;
  float l = 0.f;
  if (n < N) {
    RowPL<PL> v, u;
    v.load(z + n * D + PL * lane);
    const float nz = sqrtf(wave_sum64(v.dot(v)));
    float d2 = 0.f;
#pragma unroll
    for (int i = 0; i < PL; ++i) {
      u.v[i] = v.v[i] / nz;
      d2 += (u.v[i] - v.v[i]) * (u.v[i] - v.v[i]);
    }
    u.store(zn + n * D + PL * lane);
    if (lane == 0) zlen[n] = nz;
    l = wave_sum64(d2);
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
template <typename T, int PL>
__global__ __launch_bounds__(256) void vq_plain_bwd_kernel(const float* __restrict__ z, const float* __restrict__ zn,
                                                           const float* __restrict__ zlen, const float* __restrict__ zq,
                                                           const T* __restrict__ dzq, const int* __restrict__ src_t,
                                                           int Tn, int64_t N, int normalize, float beta, float s,
                                                           T* __restrict__ dz, const float* __restrict__ bsum,
                                                           const float* __restrict__ bcnt,
                                                           const float* __restrict__ emb, const float* __restrict__ elen,
                                                           int K, float* __restrict__ dE) {
  constexpr int D = 64 * PL;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kb = (K + 3) / 4;
  if ((int)blockIdx.x < kb) {
    const int k = blockIdx.x * 4 + w;
    if (k >= K) return;
    RowPL<PL> e, b, d;
    e.load(emb + (int64_t)k * D + PL * lane);
    b.load(bsum + (int64_t)k * D + PL * lane);
    const float c = bcnt[k];
#pragma unroll
    for (int i = 0; i < PL; ++i) d.v[i] = s * (c * e.v[i] - b.v[i]);
    if (normalize) {
      const float dot = wave_sum64(e.dot(d));
      const float il = 1.0f / elen[k];
#pragma unroll
      for (int i = 0; i < PL; ++i) d.v[i] = (d.v[i] - e.v[i] * dot) * il;
    }
    d.store(dE + (int64_t)k * D + PL * lane);
    return;
  }
  const int64_t n = (int64_t)(blockIdx.x - kb) * 4 + w;
  if (n >= N) return;
  const int64_t o = n * D + PL * lane;
  RowPL<PL> u, q, g;
  u.load(zn + o);
  q.load(zq + o);
  const int t = (int)(n % Tn);
  const bool st = dzq && (!src_t || src_t[t] == t);
#pragma unroll
  for (int i = 0; i < PL; ++i) g.v[i] = st ? Elem<T>::ld(dzq, o + i) : 0.f;
  const float bs = beta * s;
  RowPL<PL> d;
#pragma unroll
  for (int i = 0; i < PL; ++i) d.v[i] = g.v[i] + bs * (u.v[i] - q.v[i]);
  if (normalize) {
    RowPL<PL> v;
    v.load(z + o);
#pragma unroll
    for (int i = 0; i < PL; ++i) d.v[i] += bs * (u.v[i] - v.v[i]);
    const float dot = wave_sum64(u.dot(d));
    const float il = 1.0f / zlen[n];
#pragma unroll
    for (int i = 0; i < PL; ++i) d.v[i] = (d.v[i] - u.v[i] * dot) * il - bs * (u.v[i] - v.v[i]);
  }
#pragma unroll
  for (int i = 0; i < PL; ++i) Elem<T>::st(dz, o + i, d.v[i]);
}

}  // namespace

extern "C" int vqx_vq_normalize(const float* z, int64_t n_rows, int32_t D, float* E, int32_t K, float* z_norm,
                                float* z_len, float* emb_norm, float* e_len, float* partials, float* normloss_out,
                                vqx_stream_t stream) {
  if (!vq_d_ok(D)) { set_error("vqx_vq_normalize: z_dim must be 64, 128 or 256 (got %d)", D); return -1; }
  if (!z || !E || !z_norm || !z_len || !emb_norm || !e_len || !partials || n_rows < 1 || K < 1) {
    set_error("vqx_vq_normalize: bad arguments");
    return -1;
  }
  hipStream_t s = (hipStream_t)stream;
  const int kb = (K + 3) / 4;
  const int64_t zb = (n_rows + 3) / 4;
  auto* kfn = D == 64 ? vq_normalize_kernel<1> : D == 128 ? vq_normalize_kernel<2> : vq_normalize_kernel<4>;
  hipLaunchKernelGGL(kfn, dim3((unsigned)(kb + zb)), dim3(256), 0, s, z, n_rows, E, K, z_norm, z_len, emb_norm, e_len,
                     partials);
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
  if (!vq_d_ok(D)) { set_error("vqx_vq_plain_bwd: z_dim must be 64, 128 or 256 (got %d)", D); return -1; }
  if (!z_norm || !zq || !dz || !bsum || !bcnt || !emb || !dE || T < 1 || n_rows < 1 || K < 1 ||
      (normalize && (!z || !z_len || !e_len))) {
    set_error("vqx_vq_plain_bwd: bad arguments");
    return -1;
  }
  const int kb = (K + 3) / 4;
  const int64_t zb = (n_rows + 3) / 4;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)(kb + zb));
  if (dtype == VQX_BF16) {
    auto* kfn = D == 64 ? vq_plain_bwd_kernel<bf16_t, 1> : D == 128 ? vq_plain_bwd_kernel<bf16_t, 2>
                                                                    : vq_plain_bwd_kernel<bf16_t, 4>;
    hipLaunchKernelGGL(kfn, grid, dim3(256), 0, s, z, z_norm, z_len, zq, (const bf16_t*)dzq, src_t, T, n_rows,
                       normalize, beta, scale, (bf16_t*)dz, bsum, bcnt, emb, e_len, K, dE);
  } else {
    auto* kfn = D == 64 ? vq_plain_bwd_kernel<float, 1> : D == 128 ? vq_plain_bwd_kernel<float, 2>
                                                                   : vq_plain_bwd_kernel<float, 4>;
    hipLaunchKernelGGL(kfn, grid, dim3(256), 0, s, z, z_norm, z_len, zq, (const float*)dzq, src_t, T, n_rows,
                       normalize, beta, scale, (float*)dz, bsum, bcnt, emb, e_len, K, dE);
  }
  return launch_status("vqx_vq_plain_bwd");
}
