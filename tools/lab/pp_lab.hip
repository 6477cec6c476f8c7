// Ping-pong 8-wave conv GEMM (FWD, bf16) lab: 256 x BN tile, BK = 64,
// two wave groups alternating LDS-read and MFMA phases.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <cmath>
#include <string.h>

#include "../../vae_npvc_amd/csrc/vqx_gemm_kernel.h"

namespace vqx {
void set_error(const char*, ...) {}
int launch_status(const char*) { return 0; }
}  // namespace vqx
using namespace vqx;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

#ifndef LAB
#define LAB 0
#endif

__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

// BN: 256 or 128. NB: LDS K-tile buffers. R: read phases per K-tile (1 or 2).
template <int BN, int NB, int R>
__global__ __launch_bounds__(512, 1) void pp_fwd(GemmParams P) {
  constexpr int BM = 256, BK = 64, ES = 2;
  constexpr int A_BYTES = BM * BK * ES, B_BYTES = BN * BK * ES, STAGE = A_BYTES + B_BYTES;
  constexpr int WN = BN / 4, NBC = WN / 16;        // wave tile 128 x WN, col blocks per wave
  constexpr int NBH = NBC / 2;                      // B halves (2 col blocks each)
  constexpr int NPH = 2 * NBH;                      // phases per K-tile
  constexpr int GA = A_BYTES / 8192, GB = B_BYTES / 8192, NG = GA + GB;  // glds per thread per K-tile
  constexpr int GPP = (NG + NPH - 1) / NPH;         // glds per issue phase (a tile's window = NPH phases)
  constexpr int L = NB * NPH - R;                   // issue lookahead (phases)
  static_assert(L >= NPH + 1, "pipeline too shallow");
  __shared__ __attribute__((aligned(16))) char smem[NB * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2, wc = wid & 3;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = lin / P.tiles_n, tn = lin - tm * P.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = P.K / BK;

  // glds piece g (0..NG-1) of a K-tile: pieces 0..GA-1 = A (8 KB each = 64 rows), rest B.
  // Thread t writes chunk c = g_local*512 + t  (lane-linear per wave: wave w, lane l -> 16*(w*64+l))
  unsigned aoff[GA], boff[GB];
  int amask[GA];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int c = i * 512 + tid;
    const int row = c >> 3, kch = (c & 7) ^ kswz<8>(row);
    const int64_t n = (int64_t)m0 + row;
    const int t = (int)(n % P.T);
    int msk = 0;
    if (n < P.n_rows)
      for (int j = 0; j < 3; ++j) msk |= ((t + j - P.pad >= 0) && (t + j - P.pad < P.T)) ? (1 << j) : 0;
    amask[i] = msk;
    aoff[i] = (unsigned)((n * P.lda + kch * 8) * ES + (int64_t)P.pad * P.lda * ES);
  }
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int c = i * 512 + tid;
    const int row = c >> 3, kch = (c & 7) ^ kswz<8>(row);
    const int co = n0 + row;
    boff[i] = co < P.Nc ? (unsigned)(((int64_t)co * P.K + kch * 8) * ES) : kOOB;
  }
  const __amdgpu_buffer_rsrc_t rsA = rsrc_at(P.a, -(int64_t)P.pad * P.lda * ES, P.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = rsrc_at(P.b, 0, P.b_bytes);

  auto issue = [&](int kt, int g) {  // glds piece g of K-tile kt
    const int buf = kt % NB;
    const int k0 = kt * BK;
    const int tap = k0 / P.kcin, c0 = k0 - tap * P.kcin;
    char* base = smem + buf * STAGE;
    if (g < GA) {
      const unsigned ksa = (unsigned)(((tap - P.pad) * P.lda + c0) * ES);
      const unsigned off = ((amask[g] >> tap) & 1) ? aoff[g] + ksa : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (VQX_LDS(void)*)(base + g * 8192 + wid * 1024), 16, (int)off, 0, 0, 0);
    } else {
      const int gb = g - GA;
      const unsigned off = boff[gb] + (unsigned)(k0 * ES);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (VQX_LDS(void)*)(base + A_BYTES + gb * 8192 + wid * 1024), 16, (int)off, 0, 0, 0);
    }
  };
  // phase ph (global): issue pieces of the tile whose window covers ph
  auto issue_phase = [&](int ph) {
    const int q = ph + L;            // >= 0
    const int kt = q / NPH, j = q - kt * NPH;
    if (kt < nk) {
#pragma unroll
      for (int g = 0; g < GPP; ++g)
        if (j * GPP + g < NG) issue(kt, j * GPP + g);
    }
  };
  // glds issued after tile kt's last piece and before the wait in phase kt*NPH-1
  auto inflight_at_wait = [&](int kt) {  // kt = tile being retired
    int n = 0;
    for (int ph = (kt + 1) * NPH - L; ph <= kt * NPH - 1; ++ph) {
      const int q = ph + L, t = q / NPH, j = q - t * NPH;
      if (t < nk) n += (NG - j * GPP < GPP) ? (NG - j * GPP > 0 ? NG - j * GPP : 0) : GPP;
    }
    return n;
  };

  f32x4v acc[8][NBC];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NBC; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const int l15 = lane & 15, lq = lane >> 4;
  bf16x8_t fa[2][4][2];   // [A half][row block][k-step]
  bf16x8_t fb[NBC][2];    // [col block][k-step]

  auto read_a = [&](int buf, int h) {
    const char* la = smem + buf * STAGE;
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        fa[h][rb][s] = *(const bf16x8_t*)(la + kmaj_off<8>(grp * 128 + h * 64 + rb * 16 + l15, 4 * s + lq));
  };
  auto read_b = [&](int buf) {
    const char* lb = smem + buf * STAGE + A_BYTES;
#pragma unroll
    for (int cb = 0; cb < NBC; ++cb)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        fb[cb][s] = *(const bf16x8_t*)(lb + kmaj_off<8>(wc * WN + cb * 16 + l15, 4 * s + lq));
  };
  auto mfma_q = [&](int ah, int bh) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int c = 0; c < 2; ++c)
          acc[ah * 4 + rb][bh * 2 + c] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[bh * 2 + c][s], fa[ah][rb][s], acc[ah * 4 + rb][bh * 2 + c], 0, 0, 0);
  };

  // prologue: phases -L .. -1 (issue only), retire tile 0, publish
  for (int ph = -L; ph < 0; ++ph) issue_phase(ph);
  wait_vm(inflight_at_wait(0));
  __syncthreads();
  if (grp == 1) bar();  // stagger: group 1 runs one barrier behind

  if (LAB >= 3) { read_a(0, 0); read_a(0, 1); read_b(0); }
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt % NB;
#pragma unroll
    for (int q = 0; q < NPH; ++q) {
      const int ph = kt * NPH + q;
      // ---- load part
      if (LAB >= 3) {
      } else if (q == 0) {
        read_a(buf, 0);
        read_b(buf);
        if (R == 1) read_a(buf, 1);
      } else if (q == 1 && R == 2) {
        read_a(buf, 1);
      }
#if LAB != 1 && LAB < 3
      issue_phase(ph);
#endif
      if (q == NPH - 1 && kt + 1 < nk) wait_vm(inflight_at_wait(kt + 1));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (LAB != 4) bar();
      // ---- MFMA part
      __builtin_amdgcn_sched_barrier(0);
#if LAB != 2
      __builtin_amdgcn_s_setprio(1);
      if constexpr (NPH == 4) {
        const int ah = (q < 2) ? 0 : 1, bh = (q == 0 || q == 3) ? 0 : 1;
        mfma_q(ah, bh);
      } else {
        mfma_q(q, 0);
      }
      __builtin_amdgcn_s_setprio(0);
#endif
      __builtin_amdgcn_sched_barrier(0);
      if (LAB != 4) bar();
    }
  }
  if (grp == 0) bar();  // balance the stagger

  // epilogue: accumulators -> LDS (fp32, one 128-row half per pass) -> 16-B row-contiguous bf16 stores
  constexpr int EPL = BN + 4;  // floats per staged row
  float* ep = (float*)smem;
  bf16_t* y = (bf16_t*)P.y;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    __syncthreads();
    if (grp == pass) {
#pragma unroll
      for (int rb = 0; rb < 8; ++rb)
#pragma unroll
        for (int cb = 0; cb < NBC; ++cb)
          *(f32x4v*)(ep + (rb * 16 + l15) * EPL + wc * WN + cb * 16 + 4 * lq) = acc[rb][cb];
    }
    __syncthreads();
    constexpr int CPRW = BN / 8;              // 16-B chunks per row
    constexpr int ITER = 128 * CPRW / 512;
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int c = it * 512 + tid;
      const int r = c / CPRW, cc = (c % CPRW) * 8;
      const int64_t n = (int64_t)m0 + pass * 128 + r;
      const int co = n0 + cc;
      if (n < P.n_rows && co < P.Nc) {
        const f32x4v lo = *(const f32x4v*)(ep + r * EPL + cc), hi = *(const f32x4v*)(ep + r * EPL + cc + 4);
        uint4 u;
        u.x = (unsigned)f2bf(lo[0]) | ((unsigned)f2bf(lo[1]) << 16);
        u.y = (unsigned)f2bf(lo[2]) | ((unsigned)f2bf(lo[3]) << 16);
        u.z = (unsigned)f2bf(hi[0]) | ((unsigned)f2bf(hi[1]) << 16);
        u.w = (unsigned)f2bf(hi[2]) | ((unsigned)f2bf(hi[3]) << 16);
        *(uint4*)(y + n * P.ldy + co) = u;
      }
    }
  }
}

static float bf(unsigned short v) { unsigned u = (unsigned)v << 16; float f; memcpy(&f, &u, 4); return f; }

template <int BN, int NB, int R>
static float run(const GemmParams& P, int iters) {
  const int grid = P.tiles_m * P.tiles_n;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((pp_fwd<BN, NB, R>), dim3(grid), dim3(512), 0, 0, P);
  CK(hipGetLastError());
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((pp_fwd<BN, NB, R>), dim3(grid), dim3(512), 0, 0, P);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / iters;
}

int main() {
  const int N = 16384, T = 256, iters = 50;
  struct Shape { const char* name; int cin, cout, k; };
  const Shape shapes[] = {{"dec_in_fwd", 512, 1024, 3}, {"enc_k3_fwd", 512, 512, 3}, {"enc_sk_fwd", 512, 512, 1},
                          {"dec_rs_fwd", 512, 640, 1}};
  const size_t xb = (size_t)N * 512 * 2, wb = (size_t)1024 * 3 * 512 * 2, yb = (size_t)N * 1024 * 2;
  void *x, *w, *y;
  CK(hipMalloc(&x, xb)); CK(hipMalloc(&w, wb)); CK(hipMalloc(&y, yb));
  std::vector<unsigned short> hx(xb / 2), hw(wb / 2);
  srand(1);
  for (auto& v : hx) v = (unsigned short)(0x3c00 + (rand() % 0x300)) ^ ((rand() & 1) << 15);
  for (auto& v : hw) v = (unsigned short)(0x3c00 + (rand() % 0x300)) ^ ((rand() & 1) << 15);
  CK(hipMemcpy(x, hx.data(), xb, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, hw.data(), wb, hipMemcpyHostToDevice));
  std::vector<unsigned short> hy((size_t)N * 1024);
  for (const Shape& s : shapes) {
    GemmParams P = {};
    P.T = T; P.n_rows = N; P.ntaps = s.k; P.pad = (s.k - 1) / 2; P.sign = 1; P.y = y;
    P.a = x; P.b = w; P.lda = s.cin; P.kcin = s.cin; P.K = s.k * s.cin; P.Mc = N; P.Nc = s.cout;
    P.a_bytes = (int64_t)N * s.cin * 2; P.b_bytes = (int64_t)s.k * s.cin * s.cout * 2;
    P.cdim = s.cout; P.ldy = s.cout;
    const double flops = 2.0 * N * s.cin * s.cout * s.k;
    float t256 = -1, t128a = -1, t128b = -1;
    double e256 = -1, e128a, e128b;
    P.tiles_m = N / 256;
    auto verify = [&]() {
    CK(hipMemcpy(hy.data(), y, (size_t)N * s.cout * 2, hipMemcpyDeviceToHost));
    CK(hipMemset(y, 0xff, (size_t)N * s.cout * 2));
    double maxerr = 0;
    for (int probe = 0; probe < 64; ++probe) {
      const int n = (probe * 2654435761u) % N, co = (probe * 40503u) % s.cout, t = n % T;
      double ref = 0;
      for (int j = 0; j < s.k; ++j) {
        const int tt = t + j - P.pad;
        if (tt < 0 || tt >= T) continue;
        for (int ci = 0; ci < s.cin; ++ci)
          ref += (double)bf(hx[(size_t)(n + j - P.pad) * s.cin + ci]) * bf(hw[(size_t)co * P.K + j * s.cin + ci]);
      }
      const double got = bf(hy[(size_t)n * s.cout + co]);
      maxerr = fmax(maxerr, fabs(got - ref) / (fabs(ref) + 1.0));
    }
    return maxerr;
    };
    if (s.cout % 256 == 0) { P.tiles_n = s.cout / 256; t256 = run<256, 2, 2>(P, iters); e256 = verify(); }
    P.tiles_n = (s.cout + 127) / 128;
    t128a = run<128, 3, 2>(P, iters);
    e128a = verify();
    t128b = run<128, 3, 1>(P, iters);
    e128b = verify();
    printf("lab%d %-12s 256x256: %6.1f us %6.0f TF | 256x128 R2: %6.1f us %6.0f TF | R1: %6.1f us %6.0f TF | err %.1e %.1e %.1e\n",
           LAB, s.name, t256, t256 > 0 ? flops / t256 / 1e6 : 0.0, t128a, flops / t128a / 1e6, t128b, flops / t128b / 1e6,
           e256, e128a, e128b);
  }
  return 0;
}
