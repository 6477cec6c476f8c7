// Stand-alone timing lab for the tap-reuse conv kernels (conv_tr_kernel,
// conv_tr8_kernel, wgrad_tr_kernel) at the config-2 3-tap shapes.  Built per variant with
// -DVQX_GEMM_LAB=0..3 (full / no operand DMA / no MFMA / no epilogue) by
// tools/lab/tr_lab.sh; prints the mean launch time over 20 launches.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <algorithm>
#include <vector>

#include "vqx_gemm_kernel.h"
#include "vqx_gemm_pp.h"
#ifndef VQX_GEMM_LAB
#define VQX_GEMM_LAB VQX_PP_LAB
#endif

using namespace vqx;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

struct Shape {
  const char* name;
  int mode;
  int64_t N;
  int T, kin, kout;
};

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

static float bf2f(unsigned short v) {
  unsigned u = (unsigned)v << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// one launch of `fn` vs one of conv_tr_kernel (the tested kernel) on the same inputs: max |diff| / max |ref|
static void check(const Shape& s, const char* name, const void* fn, int rows, int block, GemmParams P) {
  const size_t n = (size_t)s.N * s.kout;
  std::vector<unsigned short> a(n), b(n);
  void* args[] = {(void*)&P};
  CK(hipMemset(P.y, 0, n * 2));
  CK(hipLaunchKernel(fn, dim3(P.tiles_m * P.tiles_n), dim3(block), args, 0, 0));
  CK(hipMemcpy(a.data(), P.y, n * 2, hipMemcpyDeviceToHost));
  GemmParams R = P;
  R.tiles_m = (int)(s.N / 128);
  void* rargs[] = {(void*)&R};
  CK(hipMemset(P.y, 0, n * 2));
  const void* ref = s.mode == MODE_FWD ? (const void*)conv_tr_kernel<MODE_FWD, EK_NONE, 32>
                                       : (const void*)conv_tr_kernel<MODE_DGRAD, EK_NONE, 32>;
  CK(hipLaunchKernel(ref, dim3(R.tiles_m * R.tiles_n), dim3(256), rargs, 0, 0));
  CK(hipMemcpy(b.data(), P.y, n * 2, hipMemcpyDeviceToHost));
  double mx = 0, md = 0;
  size_t nbad = 0;
  for (size_t i = 0; i < n; ++i) {
    const double x = bf2f(a[i]), y = bf2f(b[i]);
    mx = std::max(mx, std::fabs(y));
    md = std::max(md, std::fabs(x - y));
    if (std::fabs(x - y) > 1e-2 * std::fabs(y) + 1e-3) ++nbad;
  }
  printf("check %-13s %-10s maxdiff/maxref %.3e  bad %zu of %zu\n", s.name, name, md / mx, nbad, n);
}

template <int MODE, int EK>
static void run(const Shape& s, void* x, void* w, void* y, float* part) {
  GemmParams P = {};
  P.a = x;
  P.b = w;
  P.a_bytes = ((s.N - 1) * (int64_t)s.kin + s.kin) * 2;
  P.b_bytes = (int64_t)3 * s.kin * s.kout * 2;
  P.n_rows = s.N;
  P.T = s.T;
  P.lda = s.kin;
  P.kcin = s.kin;
  P.K = 3 * s.kin;
  P.Mc = (int)s.N;
  P.Nc = s.kout;
  P.ntaps = 3;
  P.pad = 1;
  P.sign = 1;
  P.dil = 1;
  P.cdim = s.kout;
  P.tiles_n = s.kout / 128;
  P.splits = 1;
  P.y = y;
  P.ldy = s.kout;
  P.epi = EK == EK_GNSTATS ? VQX_EPI_GNSTATS : 0;
  P.stat_part = part;
  P.gn_groups = s.kout > 512 ? 2 : s.kout / 128;
  const double fl = 2.0 * s.N * s.kout * 3.0 * s.kin;
  struct V {
    const char* name;
    const void* fn;
    int rows, block;
  } vs[] = {{"tr128", (const void*)conv_tr_kernel<MODE, EK, 32>, 128, 256},
            {"tr8x256", (const void*)conv_tr8_kernel<MODE, EK, 1>, 256, 512},
            {"tr8x512", (const void*)conv_tr8_kernel<MODE, EK, 2>, 512, 512},
            {"pp512u2", (const void*)conv_pp_kernel<MODE, EK, 2, 2>, 512, 512},
            {"pp256u1", (const void*)conv_pp_kernel<MODE, EK, 1, 1>, 256, 512},
            {"pp512m16", MODE == MODE_FWD ? (const void*)conv_pp_kernel<MODE_FWD, EK, 2, 3, true> : nullptr, 512, 512},
            {"pp256m16", MODE == MODE_FWD ? (const void*)conv_pp_kernel<MODE_FWD, EK, 1, 3, true> : nullptr, 256, 512},
            {"pp256u2", (const void*)conv_pp_kernel<MODE, EK, 1, 2>, 256, 512}};
  for (const V& v : vs) {
    if (!v.fn) continue;
    P.tiles_m = (int)(s.N / v.rows);
    if (getenv("TR_LAB_CHECK")) check(s, v.name, v.fn, v.rows, v.block, P);
    const float us = time_us(v.fn, P.tiles_m * P.tiles_n, v.block, P, 20);
    printf("lab%d %-13s EK%d %-10s %7.1f us %7.1f TF\n", VQX_GEMM_LAB, s.name, EK, v.name, us, fl / us * 1e-6);
  }
}

// wgrad_tr_kernel: S[r][j*c + cc] over split-K slabs (bf16 slabs, as the bf16 step)
static void run_wgrad(const char* name, int64_t N, int T, int r_dim, int c_dim, int splits, int sign, void* p, void* q,
                      void* slabs) {
  GemmParams P = {};
  P.a = p;
  P.b = q;
  P.n_rows = N;
  P.T = T;
  P.lda = r_dim;
  P.ldb = c_dim;
  P.a_bytes = N * r_dim * 2;
  P.b_bytes = N * c_dim * 2;
  P.Mc = r_dim;
  P.Nc = 3 * c_dim;
  P.ntaps = 3;
  P.pad = 1;
  P.sign = sign;
  P.dil = 1;
  P.cdim = c_dim;
  P.splits = splits;
  P.k_per_split = (N + splits - 1) / splits;
  P.k_per_split = (P.k_per_split + 63) / 64 * 64;
  P.y = slabs;
  P.slab_bf16 = 1;
  P.tap_reuse = 1;
  P.tiles_m = (r_dim + 127) / 128;
  P.tiles_n = c_dim / 64;
  const double fl = 2.0 * N * r_dim * 3.0 * c_dim;
  const float us = time_us((const void*)wgrad_tr_kernel<EK_NONE>, P.tiles_m * P.tiles_n * splits, 256, P, 20);
  printf("lab%d %-13s wgrad_tr s%-2d      %7.1f us %7.1f TF\n", VQX_GEMM_LAB, name, splits, us, fl / us * 1e-6);
}

int main() {
  const Shape shapes[] = {{"dec_in_fwd", MODE_FWD, 16384, 256, 512, 1024},
                          {"enc_k3_fwd", MODE_FWD, 16384, 256, 512, 512},
                          {"dec_in_dgrad", MODE_DGRAD, 16384, 256, 1024, 512},
                          {"enc_k3_dgrad", MODE_DGRAD, 16384, 256, 512, 512}};
  const size_t xb = (size_t)16384 * 1024 * 2, wb = (size_t)3 * 1024 * 1024 * 2;
  std::vector<unsigned short> h(xb / 2);
  unsigned r = 12345u;
  for (auto& v : h) {
    r = r * 1664525u + 1013904223u;
    v = (unsigned short)(0x3c00 + ((r >> 16) & 0x7f) - 0x40) | ((r & 1) << 15);  // small bf16 values
  }
  void *x, *w, *y;
  float* part;
  CK(hipMalloc(&x, xb));
  CK(hipMalloc(&w, wb));
  CK(hipMalloc(&y, xb));
  CK(hipMalloc(&part, (size_t)128 * 8 * 4 * 4));
  CK(hipMemcpy(x, h.data(), xb, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, h.data(), wb, hipMemcpyHostToDevice));
  CK(hipMemcpy(y, h.data(), xb, hipMemcpyHostToDevice));  // wgrad's q operand
  if (!getenv("TR_LAB_SKIP_WGRAD")) {
    void* sl;
    CK(hipMalloc(&sl, (size_t)32 * 1024 * 3 * 1024 * 2));
    run_wgrad("dec_in_wgrad", 16384, 256, 512, 1024, 8, -1, x, y, sl);
    run_wgrad("enc_k3_wgrad", 16384, 256, 512, 512, 16, 1, x, y, sl);
    run_wgrad("dec_in_wgrad", 16384, 256, 512, 1024, 4, -1, x, y, sl);
    run_wgrad("dec_in_wgrad", 16384, 256, 512, 1024, 16, -1, x, y, sl);
    CK(hipFree(sl));
  }
  if (const char* e = getenv("TR_LAB_WGRAD_ONLY"); e && *e) return 0;
  for (const Shape& s : shapes) {
    if (s.mode == MODE_FWD) {
      run<MODE_FWD, EK_NONE>(s, x, w, y, part);
      run<MODE_FWD, EK_GNSTATS>(s, x, w, y, part);
    } else {
      run<MODE_DGRAD, EK_NONE>(s, x, w, y, part);
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
