// Diagnostic build: per-workgroup phase times of the 1x1 conv GEMMs (s_memtime
// Needs the stamp points of tools/lab/k1_stamp.patch applied to
// vae_npvc_amd/csrc/vqx_gemm_kernel.h (git apply tools/lab/k1_stamp.patch).
// stamps in conv_gemm_body, -DVQX_STAMP) at the config-2 shapes.  For one launch
// (after warm-ups) prints, per case: the effective clock, and over workgroups
// the median / p10 / p90 of start, end of prologue, end of main loop, end of
// epilogue relative to the earliest start, in microseconds at that clock.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define VQX_STAMP 1
#include "vqx_gemm_kernel.h"

using namespace vqx;
#ifndef K1_BK
#define K1_BK 64
#define K1_NST 2
#endif

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

static void* dmalloc(size_t bytes, const std::vector<unsigned short>& h) {
  void* p;
  CK(hipMalloc(&p, bytes));
  CK(hipMemcpy(p, h.data(), bytes < h.size() * 2 ? bytes : h.size() * 2, hipMemcpyHostToDevice));
  return p;
}

static double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(q * (v.size() - 1))];
}

int main() {
  const int64_t N = 16384;
  const int T = 256, B = 64;
  std::vector<unsigned short> h((size_t)N * 1024);
  unsigned r = 12345u;
  for (auto& v : h) {
    r = r * 1664525u + 1013904223u;
    v = (unsigned short)(0x3c00 + ((r >> 16) & 0x7f) - 0x40) | ((r & 1) << 15);
  }
  std::vector<unsigned short> hf(8 * 1024);
  for (size_t i = 0; i < hf.size(); i += 2) { hf[i] = 0; hf[i + 1] = 0x3f80; }
  void* x = dmalloc((size_t)N * 1024 * 2, h);
  void* w = dmalloc((size_t)1024 * 1024 * 2, h);
  void* y = dmalloc((size_t)N * 1024 * 2, h);
  void* y2 = dmalloc((size_t)N * 1024 * 2, h);
  void* gnh = dmalloc((size_t)N * 1024 * 2, h);
  void* res = dmalloc((size_t)N * 1024 * 2, h);
  float* o2 = (float*)dmalloc((size_t)N * 128 * 4, h);
  float* vec = (float*)dmalloc(hf.size() * 2, hf);
  float* mr = (float*)dmalloc(hf.size() * 2, hf);
  float* part = (float*)dmalloc((size_t)(N / 128) * 1024 * 4, h);
  {
    std::vector<float> m(4 * B);
    for (int i = 0; i < 4 * B; ++i) m[i] = (i & 1) ? 1.f : 0.f;
    CK(hipMemcpy(mr, m.data(), m.size() * 4, hipMemcpyHostToDevice));
  }
  unsigned long long* sb;
  CK(hipMalloc(&sb, 8192 * 8 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(vqx_stamp_buf), &sb, sizeof(sb)));
  struct Case {
    const char* name;
    int mode, kin, kout, epi, ek;
  } cases[] = {
      {"enc_sk_fwd GNADD+ACT2", MODE_FWD, 512, 512, VQX_EPI_BIAS | VQX_EPI_GNADD | VQX_EPI_ACT2, EK_GNADD},
      {"enc_sk_fwd plain", MODE_FWD, 512, 512, 0, EK_NONE},
      {"dec_rs_fwd RES+SPLIT", MODE_FWD, 512, 640, VQX_EPI_BIAS | VQX_EPI_RES | VQX_EPI_SPLIT, EK_SPLIT},
      {"dec_rs_dgrad GNBWD", MODE_DGRAD, 640, 512, VQX_EPI_GNBWD, EK_GNBWD},
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
    P.ldgn = c.kin == 640 ? 1024 : 512;
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
    const void* fn;
    if (c.mode == MODE_FWD) {
      if (c.ek == EK_GNADD) fn = (const void*)conv_gemm_kernel<bf16_t, MODE_FWD, VQX_PRO_NONE, false, K1_BK, K1_NST, EK_GNADD>;
      else if (c.ek == EK_SPLIT) fn = (const void*)conv_gemm_kernel<bf16_t, MODE_FWD, VQX_PRO_NONE, false, K1_BK, K1_NST, EK_SPLIT>;
      else fn = (const void*)conv_gemm_kernel<bf16_t, MODE_FWD, VQX_PRO_NONE, false, K1_BK, K1_NST, EK_NONE>;
    } else {
      fn = (const void*)conv_gemm_kernel<bf16_t, MODE_DGRAD, VQX_PRO_NONE, false, K1_BK, K1_NST, EK_GNBWD>;
    }
    const int grid = P.tiles_m * P.tiles_n;
#ifdef K1_THREE
    if (c.ek == EK_SPLIT) fn = (const void*)conv_gemm3_kernel<bf16_t, MODE_FWD, VQX_PRO_NONE, false, EK_SPLIT>;
    else if (c.ek == EK_GNADD) fn = (const void*)conv_gemm3_kernel<bf16_t, MODE_FWD, VQX_PRO_NONE, false, EK_GNADD>;
    else if (c.mode == MODE_FWD) fn = (const void*)conv_gemm3_kernel<bf16_t, MODE_FWD, VQX_PRO_NONE, false, EK_NONE>;
    else fn = (const void*)conv_gemm3_kernel<bf16_t, MODE_DGRAD, VQX_PRO_NONE, false, EK_GNBWD>;
    printf("three/CU ");
#endif
    void* args[] = {(void*)&P};
    for (int i = 0; i < 10; ++i) CK(hipLaunchKernel(fn, dim3(grid), dim3(256), args, 0, 0));
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> st((size_t)grid * 8);
    CK(hipMemcpy(st.data(), sb, st.size() * 8, hipMemcpyDeviceToHost));
    // memtime bases differ between XCDs: durations from memtime deltas within a
    // workgroup, placement in time from the 100 MHz realtime stamps
    unsigned long long r0 = ~0ull;
    for (int b = 0; b < grid; ++b) r0 = std::min(r0, st[b * 8 + 4]);
    std::vector<double> clk, beg, fin, d[3];
    for (int b = 0; b < grid; ++b) {
      const unsigned long long* o = &st[b * 8];
      const double rt = (double)(o[5] - o[4]) * 10.0;  // ns
      clk.push_back(rt > 0 ? (double)(o[3] - o[0]) / rt : 0.0);
      beg.push_back((o[4] - r0) / 100.0);
      fin.push_back((o[5] - r0) / 100.0);
    }
    const double ghz = pct(clk, 0.5);
    for (int b = 0; b < grid; ++b)
      for (int i = 0; i < 3; ++i) d[i].push_back((st[b * 8 + i + 1] - st[b * 8 + i]) / (ghz * 1e3));
    printf("bk%d nst%d ", K1_BK, K1_NST);
    printf("%-22s grid %4d clock %.2f GHz  last end %.1f us\n", c.name, grid, ghz, pct(fin, 1.0));
    printf("   %-13s at  p10 %6.1f  p50 %6.1f  p90 %6.1f  max %6.1f us\n", "start", pct(beg, 0.1), pct(beg, 0.5),
           pct(beg, 0.9), pct(beg, 1.0));
    printf("   %-13s at  p10 %6.1f  p50 %6.1f  p90 %6.1f  max %6.1f us\n", "end", pct(fin, 0.1), pct(fin, 0.5),
           pct(fin, 0.9), pct(fin, 1.0));
    const char* dn[3] = {"prologue", "main loop", "epilogue"};
    for (int i = 0; i < 3; ++i)
      printf("   %-13s len p10 %6.1f  p50 %6.1f  p90 %6.1f  max %6.1f us\n", dn[i], pct(d[i], 0.1), pct(d[i], 0.5),
             pct(d[i], 0.9), pct(d[i], 1.0));
  }
  return 0;
}
