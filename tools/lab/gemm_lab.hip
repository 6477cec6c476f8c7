// Stand-alone conv-GEMM microbenchmark (no torch): times one kernel variant on
// the config-2 layer shapes.  Built per lab mode by tools/lab/build.sh:
//   VQX_LAB_MODE 0 = the production kernel, 1 = no operand DMA in the main
//   loop (MFMA + LDS reads + barriers only), 2 = no MFMA (staging only).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../vae_npvc_amd/csrc/vqx_gemm_kernel.h"

namespace vqx {
void set_error(const char*, ...) {}
int launch_status(const char*) { return 0; }
}  // namespace vqx
using namespace vqx;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <int MODE, int BK, int NST>
static float run(const GemmParams& P0, int grid, int iters) {
  GemmParams P = P0;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((conv_gemm_kernel<bf16_t, MODE, 0, false, BK, NST>), dim3(grid), dim3(256), 0, 0, P);
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((conv_gemm_kernel<bf16_t, MODE, 0, false, BK, NST>), dim3(grid), dim3(256), 0, 0, P);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / iters;
}

int main(int argc, char** argv) {
  const int N = 16384, T = 256, iters = 50;
  struct Shape { const char* name; int mode, cin, cout, k; };
  const Shape shapes[] = {{"dec_in_fwd", MODE_FWD, 512, 1024, 3}, {"enc_k3_fwd", MODE_FWD, 512, 512, 3},
                          {"enc_sk_fwd", MODE_FWD, 512, 512, 1}, {"dec_in_dgrad", MODE_DGRAD, 1024, 512, 3},
                          {"dec_in_wgrad", MODE_WGRAD, 512, 1024, 3},
                          {"k64", MODE_FWD, 64, 512, 1}, {"k128", MODE_FWD, 128, 512, 1},
                          {"k256", MODE_FWD, 256, 512, 1}, {"k512", MODE_FWD, 512, 512, 1},
                          {"k1024", MODE_FWD, 1024, 512, 1}, {"k1536", MODE_FWD, 1536, 512, 1}};
  void *x, *w, *y;
  const size_t xb = (size_t)N * 1536 * 2, wb = (size_t)1536 * 3 * 1024 * 2, yb = (size_t)8 * 1024 * 3 * 1024 * 4;
  CK(hipMalloc(&x, xb)); CK(hipMalloc(&w, wb)); CK(hipMalloc(&y, yb));
  std::vector<unsigned short> hx(xb / 2);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = 0x3f80 ^ (unsigned short)((i * 2654435761u) >> 20 & 0x807f);
  CK(hipMemcpy(x, hx.data(), xb, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, hx.data(), wb, hipMemcpyHostToDevice));
  for (const Shape& s : shapes) {
    GemmParams P = {};
    P.T = T; P.n_rows = N; P.ntaps = s.k; P.pad = (s.k - 1) / 2; P.sign = 1; P.y = y;
    int grid;
    const int mult = 1;
    (void)mult;
    if (s.mode != MODE_WGRAD) {
      P.a = x; P.b = w; P.lda = s.cin; P.kcin = s.cin; P.K = s.k * s.cin; P.Mc = N; P.Nc = s.cout;
      P.a_bytes = (int64_t)N * s.cin * 2; P.b_bytes = (int64_t)s.k * s.cin * s.cout * 2;
      P.cdim = s.cout; P.ldy = s.cout; P.tiles_n = (s.cout + 127) / 128; P.tiles_m = N / 128;
      grid = P.tiles_m * P.tiles_n;
    } else {
      const int splits = 5;
      P.a = x; P.b = x; P.lda = s.cout; P.ldb = s.cin;  // p = dy [N][cout], q = x [N][cin] (both inside x)
      P.a_bytes = (int64_t)N * s.cout * 2; P.b_bytes = (int64_t)N * s.cin * 2;
      P.Mc = s.cout; P.Nc = s.k * s.cin; P.cdim = s.cin; P.tiles_n = (P.Nc + 127) / 128; P.tiles_m = (s.cout + 127) / 128;
      P.splits = splits; P.k_per_split = ((N + splits - 1) / splits + 63) / 64 * 64;
      grid = P.tiles_m * P.tiles_n * splits;
    }
    const double flops = 2.0 * N * s.cin * s.cout * s.k;
    float us1, us2;
    if (s.mode == MODE_FWD) { us1 = run<MODE_FWD, 64, 2>(P, grid, iters); us2 = run<MODE_FWD, 32, 4>(P, grid, iters); }
    else if (s.mode == MODE_DGRAD) { us1 = run<MODE_DGRAD, 64, 2>(P, grid, iters); us2 = run<MODE_DGRAD, 32, 4>(P, grid, iters); }
    else { us1 = run<MODE_WGRAD, 64, 2>(P, grid, iters); us2 = run<MODE_WGRAD, 32, 4>(P, grid, iters); }
    printf("mode%d %-14s bk64x2 %7.1f us %7.1f TF   bk32x4 %7.1f us %7.1f TF\n", VQX_LAB_MODE, s.name, us1,
           flops / us1 / 1e6, us2, flops / us2 / 1e6);
  }
  return 0;
}
