// Stand-alone timing lab for the 1x1 conv GEMMs of config 2 (conv_gemm_kernel
// with the engine's fused epilogues).  Built per variant by tools/lab/k1_lab.sh
// with -DVQX_GEMM_STAGGER=n (the second half of the grid sleeps n x ~3.5 us
// before its main loop, so the two workgroups resident on a CU run their main
// loops and epilogues out of phase) and -DVQX_LAB_MODE=m (1 no operand DMA,
// 2 no MFMA, 3 no epilogue) and -DVQX_EPI_PREFETCH=0 (epilogue row operands
// loaded pass by pass instead of prefetched with the prologue).  Prints the mean launch time over 20 launches.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef VQX_LAB_MODE
#define VQX_LAB_MODE 0
#endif
#include "vqx_gemm_kernel.h"
#ifndef K1_NST  // ring depth of the 64-deep K-tiles (lab: 3, 4 = one workgroup per CU)
#define K1_NST 2
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

static float time_us(const void* fn, int grid, GemmParams P, int reps) {
  void* args[] = {(void*)&P};
  for (int i = 0; i < 3; ++i) CK(hipLaunchKernel(fn, dim3(grid), dim3(256), args, 0, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) CK(hipLaunchKernel(fn, dim3(grid), dim3(256), args, 0, 0));
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  return 1e3f * ms / reps;
}

static void* dmalloc(size_t bytes, const std::vector<unsigned short>& h) {
  void* p;
  CK(hipMalloc(&p, bytes));
  CK(hipMemcpy(p, h.data(), bytes < h.size() * 2 ? bytes : h.size() * 2, hipMemcpyHostToDevice));
  return p;
}

int main() {
  const int64_t N = 16384;
  const int T = 256, B = 64;
  std::vector<unsigned short> h((size_t)N * 1024);
  unsigned r = 12345u;
  for (auto& v : h) {
    r = r * 1664525u + 1013904223u;
    v = (unsigned short)(0x3c00 + ((r >> 16) & 0x7f) - 0x40) | ((r & 1) << 15);  // bf16 in +-[0.75, 1.25)
  }
  std::vector<unsigned short> hf(8 * 1024);  // float buffers: gamma/beta/bias/mean-rstd = 1.0f-ish pairs
  for (size_t i = 0; i < hf.size(); i += 2) { hf[i] = 0; hf[i + 1] = 0x3f80; }
  void* x = dmalloc((size_t)N * 1024 * 2, h);
  void* w = dmalloc((size_t)1024 * 1024 * 2, h);
  void* y = dmalloc((size_t)N * 1024 * 2, h);
  void* y2 = dmalloc((size_t)N * 1024 * 2, h);
  void* gnh = dmalloc((size_t)N * 1024 * 2, h);
  void* res = dmalloc((size_t)N * 1024 * 2, h);
  float* o2 = (float*)dmalloc((size_t)N * 128 * 4, h);
  float* vec = (float*)dmalloc(hf.size() * 2, hf);  // bias / gamma / beta (1.0)
  float* mr = (float*)dmalloc(hf.size() * 2, hf);   // mean / rstd pairs (0, 1)
  float* part = (float*)dmalloc((size_t)(N / 128) * 1024 * 4, h);
  CK(hipMemset(mr, 0, 4 * B * 4));
  {
    std::vector<float> m(4 * B);
    for (int i = 0; i < 4 * B; ++i) m[i] = (i & 1) ? 1.f : 0.f;
    CK(hipMemcpy(mr, m.data(), m.size() * 4, hipMemcpyHostToDevice));
  }
  struct Case {
    const char* name;
    int mode, kin, kout, epi, ek;
  } cases[] = {
      {"enc_sk_fwd GNADD", MODE_FWD, 512, 512, VQX_EPI_BIAS | VQX_EPI_GNADD | VQX_EPI_ACT2, EK_GNADD},
      {"dec_rs_fwd SPLIT", MODE_FWD, 512, 640, VQX_EPI_BIAS | VQX_EPI_RES | VQX_EPI_SPLIT, EK_SPLIT},
      {"dec_rs_dgrad GNBWD", MODE_DGRAD, 640, 512, VQX_EPI_GNBWD, EK_GNBWD},
      {"enc_sk_dgrad GNBWD", MODE_DGRAD, 512, 512, VQX_EPI_GNBWD | VQX_EPI_COLSUM | VQX_EPI_RES, EK_GNBWD},
      {"enc_sk_fwd plain", MODE_FWD, 512, 512, 0, EK_NONE},
  };
  for (const Case& c : cases) {
    GemmParams P = {};
    P.a = x;
    P.b = w;
    P.a_bytes = (int64_t)N * c.kin * 2;
    P.b_bytes = (int64_t)c.kin * c.kout * 2;
    P.n_rows = N;
    P.T = T;
    P.lda = c.kin;
    P.kcin = c.kin;
    P.K = c.kin;
    P.Mc = (int)N;
    P.Nc = c.kout;
    P.ntaps = 1;
    P.pad = 0;
    P.sign = 1;
    P.dil = 1;
    P.cdim = c.kout;
    P.tiles_n = (c.kout + 127) / 128;
    P.tiles_m = (int)(N / 128);
    P.splits = 1;
    P.y = y;
    P.ldy = (c.epi & VQX_EPI_SPLIT) ? 512 : c.kout;
    P.epi = c.epi;
    P.bias = vec;
    P.res = res;
    P.ldres = 512;
    P.gn_h = gnh;
    P.ldgn = c.ek == EK_GNBWD && c.kout == 512 && c.kin == 640 ? 1024 : 512;
    P.gn_mr = mr;
    P.gn_gamma = vec;
    P.gn_beta = vec;
    P.out2 = o2;
    P.ldo2 = 128;
    P.split_col = 512;
    P.out2_acc = 1;
    P.y2 = y2;
    P.ldy2 = 512;
    P.epi_act = VQX_PRO_LRELU;
    P.colsum_part = part;
    P.stat_part = part;
    P.gn_groups = c.kin == 640 ? 2 : 1;
    P.gn_glu = c.kin == 640 ? 1 : 0;
    const void* fn = nullptr;
    if (c.mode == MODE_FWD) {
      if (c.ek == EK_GNADD) fn = (const void*)conv_gemm_kernel<bf16_t, MODE_FWD, VQX_PRO_NONE, false, 64, K1_NST, EK_GNADD>;
      else if (c.ek == EK_SPLIT) fn = (const void*)conv_gemm_kernel<bf16_t, MODE_FWD, VQX_PRO_NONE, false, 64, K1_NST, EK_SPLIT>;
      else fn = (const void*)conv_gemm_kernel<bf16_t, MODE_FWD, VQX_PRO_NONE, false, 64, K1_NST, EK_NONE>;
    } else {
      fn = (const void*)conv_gemm_kernel<bf16_t, MODE_DGRAD, VQX_PRO_NONE, false, 64, K1_NST, EK_GNBWD>;
    }
    const float us = time_us(fn, P.tiles_m * P.tiles_n, P, 20);
    const double fl = 2.0 * N * c.kin * c.kout;
#ifndef VQX_GEMM_STAGGER
#define VQX_GEMM_STAGGER 0
#endif
#ifndef VQX_EPI_PREFETCH
#define VQX_EPI_PREFETCH 1
#endif
#ifndef VQX_EPI_PREVEC_DGRAD
#define VQX_EPI_PREVEC_DGRAD 0
#endif
    printf("nst%d prevec_dgrad%d prefetch%d/dgrad%d/late%d/slab%d stagger%d mode%d %-20s %7.1f us %7.1f TF\n", K1_NST,
           VQX_EPI_PREVEC_DGRAD, VQX_EPI_PREFETCH, VQX_EPI_PREFETCH_DGRAD, VQX_EPI_PREFETCH_LATE, VQX_EPI_SLAB_PREFETCH, VQX_GEMM_STAGGER,
           VQX_LAB_MODE, c.name, us, fl / us * 1e-6);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
