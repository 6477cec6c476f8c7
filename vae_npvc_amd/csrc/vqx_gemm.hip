// Conv GEMM host side: argument checks, pipeline-variant choice, launch
// probe and the C-ABI entry points (vqx_conv1d_fwd/dgrad/wgrad).  The kernel
// is vqx_gemm_kernel.h; its instantiations live in vqx_gemm_{fwd,dgrad,wgrad}.hip.
#include <hip/hip_ext.h>
#include <stdlib.h>

#include <vector>

#include "vqx_gemm_inst.h"

namespace vqx {

// ---------------- launch probe (bench.py's roofline leg)
// While enabled, every conv GEMM is launched with hipExtLaunchKernelGGL and a
// start/stop event pair that the runtime stamps on the kernel's own dispatch
// packet, so the measured duration is the kernel's (no extra queue packets
// between kernels).  Events come from a pool reused across probe sessions.
// The probe state is per host thread (thread_local): a measurement session on
// one thread never changes another thread's launches.
struct ProbeRec {
  hipEvent_t start, stop;
  int info[5];  // dtype, mode, prologue, gen, epilogue kind
  double flops;
};
static thread_local bool g_probe_on = false;
static thread_local bool g_probe_sel_on = false;  // record only launches whose info equals g_probe_sel
static thread_local int g_probe_sel[5];
static thread_local std::vector<ProbeRec> g_probe;
static thread_local std::vector<std::pair<hipEvent_t, hipEvent_t>> g_event_pool;
static thread_local size_t g_probe_used = 0;

void gemm_launch(const void* fn, int grid, hipStream_t s, const GemmParams& P, const int info[5], double flops,
                 int block) {
  void* args[] = {(void*)&P};
  gemm_launch_args(fn, grid, s, args, info, flops, block);
}

void gemm_launch_args(const void* fn, int grid, hipStream_t s, void** args, const int info[5], double flops,
                      int block) {
  bool rec = g_probe_on;
  if (rec && g_probe_sel_on)
    for (int i = 0; i < 5; ++i) rec = rec && info[i] == g_probe_sel[i];
  if (!rec) {
    (void)hipLaunchKernel(fn, dim3(grid), dim3(block), args, 0, s);
    return;
  }
  if (g_probe_used == g_event_pool.size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
      (void)hipLaunchKernel(fn, dim3(grid), dim3(block), args, 0, s);
      return;
    }
    g_event_pool.emplace_back(a, b);
  }
  auto ev = g_event_pool[g_probe_used++];
  ProbeRec r;
  r.start = ev.first;
  r.stop = ev.second;
  for (int i = 0; i < 5; ++i) r.info[i] = info[i];
  r.flops = flops;
  g_probe.push_back(r);
  (void)hipExtLaunchKernel(fn, dim3(grid), dim3(block), args, 0, s, ev.first, ev.second, 0);
}

int cu_count() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  static thread_local int cached_dev = -1, cached = 0;  // one device per thread in practice; re-query on a switch
  if (dev != cached_dev) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 0;
    cached_dev = dev;
    cached = n;
  }
  return cached;
}

bool three_per_cu(int grid, int policy) {
  const int cus = cu_count();
  if (policy == POL_AUTO) return cus > 0 && grid <= 3 * cus;
  return policy == POL_K1_2PCU && cus > 0 && grid > 2 * cus && grid <= 3 * cus;
}

static void launch_mode(GemmParams& P, int mode, int64_t rows, int extra_mult, bool bf16, bool gen, hipStream_t s) {
  // rows: extent of the tile-M dimension; extra_mult: split-K factor (WGRAD)
  P.tiles_m = (int)((rows + 127) / 128);
  const int grid = P.tiles_m * P.tiles_n * extra_mult;
  if (mode == MODE_FWD) launch_mode_dt<MODE_FWD>(P, grid, bf16, gen, s);
  else if (mode == MODE_DGRAD) launch_mode_dt<MODE_DGRAD>(P, grid, bf16, gen, s);
  else launch_mode_dt<MODE_WGRAD>(P, grid, bf16, gen, s);
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Checks the arguments and fills P (tiles_m is set by the launch); gen = the
// generic (cin % BK != 0) tile path.
static int conv_prepare(const vqx_conv_args* a, int mode, GemmParams& P, bool& gen) {
  if (!a) { set_error("vqx_conv: null args"); return -1; }
  if (a->dtype != VQX_F32 && a->dtype != VQX_BF16) { set_error("vqx_conv: bad dtype %d", a->dtype); return -1; }
  const int epc = a->dtype == VQX_BF16 ? 8 : 4;
  const int es = a->dtype == VQX_BF16 ? 2 : 4;
  const int dil = a->dil > 0 ? a->dil : 1;
  if (a->ntaps < 1 || a->ntaps > 8 || a->pad < 0 || a->pad > (a->ntaps - 1) * dil) { set_error("vqx_conv: ntaps %d / pad %d / dil %d", a->ntaps, a->pad, dil); return -1; }
  if (a->n_rows <= 0 || a->T <= 0 || a->n_rows % a->T) { set_error("vqx_conv: n_rows %lld not a multiple of T %d", (long long)a->n_rows, a->T); return -1; }
  if (a->cin <= 0 || a->cout <= 0 || a->cin % epc || a->ldx % epc || a->cin > a->ldx) { set_error("vqx_conv: cin %d / ldx %d must be multiples of %d", a->cin, a->ldx, epc); return -1; }
  if (a->cout % 8 || a->ldy % 8) { set_error("vqx_conv: cout %d / ldy %d must be multiples of 8", a->cout, a->ldy); return -1; }
  if (mode == MODE_DGRAD && a->cout % epc) { set_error("vqx_conv_dgrad: cout %d must be a multiple of %d", a->cout, epc); return -1; }
  if (!aligned16(a->x) || !aligned16(a->w)) { set_error("vqx_conv: x/w must be 16-byte aligned"); return -1; }
  if (a->prologue < 0 || a->prologue > 3 || (mode == MODE_DGRAD && a->prologue)) { set_error("vqx_conv: bad prologue %d", a->prologue); return -1; }
  const int epi = a->epilogue;
  if ((epi & VQX_EPI_BIAS) && (!a->bias || !aligned16(a->bias))) { set_error("vqx_conv: BIAS needs a 16-B aligned bias"); return -1; }
  if ((epi & VQX_EPI_ROWBIAS) && (!a->rowbias || !aligned16(a->rowbias))) { set_error("vqx_conv: ROWBIAS needs an aligned rowbias"); return -1; }
  if ((epi & VQX_EPI_RES) && (!a->res || a->ldres % 8 || !aligned16(a->res))) { set_error("vqx_conv: RES operand"); return -1; }
  if ((epi & VQX_EPI_MASK) && (!a->mask || a->ldmask % 8 || !aligned16(a->mask))) { set_error("vqx_conv: MASK operand"); return -1; }
  if ((epi & VQX_EPI_GNADD) && !(a->gn_h && a->gn_mean_rstd && a->gn_gamma && a->gn_beta && a->ldgn % 8 == 0 && aligned16(a->gn_h) && aligned16(a->gn_gamma) && aligned16(a->gn_beta))) { set_error("vqx_conv: GNADD operands"); return -1; }
  if ((epi & VQX_EPI_SPLIT) && (!a->out2 || a->split_col % 8 || a->ldo2 % 4 || !aligned16(a->out2))) { set_error("vqx_conv: SPLIT operands"); return -1; }
  if ((epi & VQX_EPI_ACT2) && (!a->y2 || a->ldy2 % 8 || !aligned16(a->y2))) { set_error("vqx_conv: ACT2 needs a 16-B aligned y2 with ldy2 %% 8 == 0"); return -1; }
  if ((epi & (VQX_EPI_ACT | VQX_EPI_ACT2)) && a->epi_act != VQX_PRO_LRELU && a->epi_act != VQX_PRO_RELU) { set_error("vqx_conv: epi_act must be LRELU or RELU"); return -1; }
  if (epi & (VQX_EPI_GNSTATS | VQX_EPI_GNBWD)) {
    const int G = a->gn_groups;
    if ((epi & VQX_EPI_GNSTATS) && (epi & VQX_EPI_GNBWD)) { set_error("vqx_conv: GNSTATS and GNBWD are exclusive"); return -1; }
    if (!a->stat_part || a->T % 128 || G < 1 || (epi & VQX_EPI_GNADD)) { set_error("vqx_conv: GN partials need stat_part, T %% 128 == 0, no GNADD"); return -1; }
    if ((epi & VQX_EPI_GNSTATS) && (a->cout % G || (a->cout / G) % 128)) { set_error("vqx_conv: GNSTATS needs cout/G %% 128 == 0"); return -1; }
    if (epi & VQX_EPI_GNBWD) {
      if (!(a->gn_h && a->gn_mean_rstd && a->gn_gamma && aligned16(a->gn_h) && aligned16(a->gn_gamma) && a->ldgn % 8 == 0)) { set_error("vqx_conv: GNBWD operands"); return -1; }
      if (a->gn_glu && (G != 2 || !a->gn_beta || !aligned16(a->gn_beta))) { set_error("vqx_conv: GNBWD glu needs G=2 and beta"); return -1; }
      if (!a->gn_glu && (a->cout % G || (a->cout / G) % 128)) { set_error("vqx_conv: GNBWD needs cout/G %% 128 == 0"); return -1; }
    }
  }
  if ((epi & VQX_EPI_COLSUM) && !a->colsum_part) { set_error("vqx_conv: COLSUM needs colsum_part [ceil(n_rows/128)][cout]"); return -1; }
  if (!a->y || !aligned16(a->y)) { set_error("vqx_conv: y must be non-null and 16-byte aligned"); return -1; }
  if (a->kernel_policy < POL_AUTO || a->kernel_policy > POL_K1_2PCU) { set_error("vqx_conv: kernel_policy %d not in 0..5", a->kernel_policy); return -1; }

  P = GemmParams{};
  P.a = a->x; P.b = a->w;
  P.a_bytes = ((a->n_rows - 1) * (int64_t)a->ldx + a->cin) * es;
  P.n_rows = a->n_rows; P.T = a->T; P.lda = a->ldx;
  P.kcin = a->cin; P.K = a->ntaps * a->cin; P.Mc = (int)a->n_rows; P.Nc = a->cout;
  P.b_bytes = (int64_t)a->ntaps * a->cin * a->cout * es;  // packed weight, either orientation
  P.ntaps = a->ntaps; P.pad = a->pad; P.sign = 1; P.dil = dil;
  P.cdim = a->cout;
  P.pro = a->prologue; P.pro_scale = a->pro_scale;
  P.tiles_n = (a->cout + kBN - 1) / kBN; P.splits = 1;  // tiles_m: launch_mode (tile height)
  P.y = a->y; P.ldy = a->ldy; P.epi = epi; P.out_f32 = (epi & VQX_EPI_OUTF32) ? 1 : 0;
  P.bias = a->bias; P.rowbias = a->rowbias; P.res = a->res; P.ldres = a->ldres;
  P.mask = a->mask; P.ldmask = a->ldmask; P.mask_slope = a->mask_slope; P.mask_scale = a->mask_scale;
  P.gn_h = a->gn_h; P.ldgn = a->ldgn; P.gn_mr = a->gn_mean_rstd; P.gn_gamma = a->gn_gamma; P.gn_beta = a->gn_beta;
  P.out2 = a->out2; P.ldo2 = a->ldo2; P.split_col = a->split_col; P.out2_acc = a->out2_accumulate;
  P.y2 = a->y2; P.ldy2 = a->ldy2; P.epi_act = a->epi_act;
  P.colsum_part = a->colsum_part;
  P.stat_part = a->stat_part; P.gn_groups = a->gn_groups; P.gn_glu = a->gn_glu;
  P.gn_tiles = a->gn_stat_tiles; P.gn_eps = a->gn_eps;
  P.policy = a->kernel_policy;
  if (P.gn_tiles && (mode != MODE_FWD || !(epi & VQX_EPI_GNADD) || a->T % 128 || a->cout % 128 ||
                     a->gn_groups != 1 || !a->gn_mean_rstd)) {
    set_error("vqx_conv: gn_stat_tiles needs FWD with GNADD, G = 1, T %% 128 == 0, cout %% 128 == 0 and gn_mean_rstd");
    return -1;
  }
  if (P.a_bytes > 0x7fffffffLL || P.b_bytes > 0x7fffffffLL) { set_error("vqx_conv: operand larger than 2 GiB"); return -1; }
  gen = (a->cin % (a->dtype == VQX_BF16 ? 64 : 32)) != 0;
  return 0;
}

static int conv_common(const vqx_conv_args* a, int mode, hipStream_t s) {
  GemmParams P;
  bool gen;
  if (conv_prepare(a, mode, P, gen)) return -1;
  launch_mode(P, mode, a->n_rows, 1, a->dtype == VQX_BF16, gen, s);
  return launch_status(mode == MODE_FWD ? "vqx_conv1d_fwd" : "vqx_conv1d_dgrad");
}

// Checks the arguments and fills P for the weight gradient (tiles_m is set by the launch)
static int wgrad_prepare(const vqx_wgrad_args* a, GemmParams& P, bool& gen) {
  if (!a) { set_error("vqx_conv1d_wgrad: null args"); return -1; }
  if (a->dtype != VQX_F32 && a->dtype != VQX_BF16) { set_error("vqx_conv1d_wgrad: bad dtype"); return -1; }
  const int epc = a->dtype == VQX_BF16 ? 8 : 4;
  const int es = a->dtype == VQX_BF16 ? 2 : 4;
  const int dil = a->dil > 0 ? a->dil : 1;
  if (a->ntaps < 1 || a->ntaps > 8 || a->pad < 0 || a->pad > (a->ntaps - 1) * dil) { set_error("vqx_conv1d_wgrad: ntaps %d / pad %d / dil %d", a->ntaps, a->pad, dil); return -1; }
  if (a->n_rows <= 0 || a->T <= 0 || a->n_rows % a->T) { set_error("vqx_conv1d_wgrad: bad n_rows/T"); return -1; }
  if (a->r_dim % epc || a->c_dim % epc || a->ldp % epc || a->ldq % epc || a->c_dim % 8) { set_error("vqx_conv1d_wgrad: dims must be multiples of %d (c_dim of 8)", epc); return -1; }
  if (a->splits < 1) { set_error("vqx_conv1d_wgrad: splits < 1"); return -1; }
  if (!aligned16(a->p) || !aligned16(a->q) || !a->slabs || !aligned16(a->slabs)) { set_error("vqx_conv1d_wgrad: bad pointers"); return -1; }
  if (a->shift_sign != 1 && a->shift_sign != -1) { set_error("vqx_conv1d_wgrad: shift_sign must be +-1"); return -1; }
  if (a->slab_dtype != VQX_F32 && !(a->slab_dtype == VQX_BF16 && a->dtype == VQX_BF16)) { set_error("vqx_conv1d_wgrad: slab_dtype %d (bf16 slabs need bf16 operands)", a->slab_dtype); return -1; }
  if (a->kernel_policy < POL_AUTO || a->kernel_policy > POL_K1_2PCU) { set_error("vqx_conv1d_wgrad: kernel_policy %d not in 0..5", a->kernel_policy); return -1; }
  P = GemmParams{};
  P.a = a->p; P.b = a->q; P.n_rows = a->n_rows; P.T = a->T; P.lda = a->ldp; P.ldb = a->ldq;
  P.a_bytes = ((a->n_rows - 1) * (int64_t)a->ldp + a->r_dim) * es;
  P.b_bytes = ((a->n_rows - 1) * (int64_t)a->ldq + a->c_dim) * es;
  if (P.a_bytes > 0x7fffffffLL || P.b_bytes > 0x7fffffffLL) { set_error("vqx_conv1d_wgrad: operand larger than 2 GiB"); return -1; }
  P.Mc = a->r_dim; P.Nc = a->ntaps * a->c_dim; P.ntaps = a->ntaps; P.pad = a->pad; P.sign = a->shift_sign; P.dil = dil;
  P.cdim = a->c_dim; P.pro = a->q_prologue; P.pro_scale = a->pro_scale;
  P.tiles_n = (P.Nc + kBN - 1) / kBN; P.splits = a->splits;  // tiles_m: launch_mode
  int64_t kps = (a->n_rows + a->splits - 1) / a->splits;
  const int kround = a->dtype == VQX_BF16 ? 64 : 32;  // whole K-tiles of either bf16 BK
  kps = (kps + kround - 1) / kround * kround;
  P.k_per_split = kps;
  P.y = a->slabs;
  P.slab_bf16 = a->slab_dtype == VQX_BF16;
  P.policy = a->kernel_policy;
  const int bkv = a->dtype == VQX_BF16 ? 64 : 32;
  gen = (a->T % bkv) != 0 || (a->n_rows % bkv) != 0;
  if (!gen && wgrad_tr_ok(a->n_rows, a->T, a->c_dim, a->ntaps, a->pad, dil, a->dtype == VQX_BF16, a->q_prologue,
                          a->kernel_policy)) {
    P.tap_reuse = 1;
    P.tiles_n = a->c_dim / 64;
  }
  if (a->fixup_dw) {  // in-launch ordered split-K reduction (ABI 127)
    if (!P.tap_reuse || !P.slab_bf16) { set_error("vqx_conv1d_wgrad: fixup_dw needs the 3-tap tap-reuse kernel and bf16 slabs (vqx_wgrad_fixup_ok)"); return -1; }
    if (!aligned16(a->fixup_dw) || !a->fixup_counters) { set_error("vqx_conv1d_wgrad: fixup_dw must be 16-B aligned, fixup_counters non-null"); return -1; }
    if ((int64_t)a->splits * P.Mc * P.Nc * 2 > 0x7fffffffLL) { set_error("vqx_conv1d_wgrad: fixup slabs larger than 2 GiB"); return -1; }
    P.fix_dw = a->fixup_dw;
    P.fix_cnt = a->fixup_counters;
  }
  return 0;
}

}  // namespace vqx

using namespace vqx;

extern "C" int vqx_conv1d_fwd(const vqx_conv_args* a, vqx_stream_t stream) {
  return conv_common(a, MODE_FWD, (hipStream_t)stream);
}

extern "C" int vqx_conv1d_dgrad(const vqx_conv_args* a, vqx_stream_t stream) {
  return conv_common(a, MODE_DGRAD, (hipStream_t)stream);
}

extern "C" int vqx_conv1d_wgrad(const vqx_wgrad_args* a, vqx_stream_t stream) {
  GemmParams P;
  bool gen;
  if (wgrad_prepare(a, P, gen)) return -1;
  launch_mode(P, MODE_WGRAD, P.Mc, P.splits, a->dtype == VQX_BF16, gen, (hipStream_t)stream);
  return launch_status("vqx_conv1d_wgrad");
}

extern "C" int vqx_conv1d_dgrad_wgrad(const vqx_conv_args* d, const vqx_wgrad_args* w, int32_t* fused,
                                      vqx_stream_t stream) {
  GemmParams PD, PW;
  bool gd, gw;
  if (conv_prepare(d, MODE_DGRAD, PD, gd)) return -1;
  if (wgrad_prepare(w, PW, gw)) return -1;
  hipStream_t s = (hipStream_t)stream;
  const bool bf = d->dtype == VQX_BF16 && w->dtype == VQX_BF16;
  // fused DGRAD + WGRAD launches unless the call keeps every GEMM on the
  // implicit-im2col kernels.  Measured (profiles/r02/dual_ab.txt): 3-tap pairs
  // interleaved 3-8% faster than two launches; 1x1 pairs in sequence 0.7% off
  // the step.  The interleaved and three-per-CU 1x1 forms measured slower and
  // were retired in round 3; WGRAD-first 1x1 pairs with fewer splits in round 4
  // (profiles/r04/slab_wfirst_ab.txt).
  if (bf && !gd && !gw && d->kernel_policy != POL_IM2COL) {
    PD.tiles_m = (int)((d->n_rows + 127) / 128);
    PW.tiles_m = (PW.Mc + 127) / 128;
    if (launch_dual(PD, PD.tiles_m * PD.tiles_n, PW, PW.tiles_m * PW.tiles_n * PW.splits, s)) {
      if (fused) *fused = 1;
      return launch_status("vqx_conv1d_dgrad_wgrad");
    }
  }
  // two launches in the engine's order: weight gradient, then data gradient
  launch_mode(PW, MODE_WGRAD, PW.Mc, PW.splits, w->dtype == VQX_BF16, gw, s);
  launch_mode(PD, MODE_DGRAD, d->n_rows, 1, d->dtype == VQX_BF16, gd, s);
  if (fused) *fused = 0;
  return launch_status("vqx_conv1d_dgrad_wgrad");
}

extern "C" int vqx_wgrad_tiles(int64_t n_rows, int32_t T, int32_t r_dim, int32_t c_dim, int32_t ntaps, int32_t pad,
                               int32_t dil, int32_t dtype, int32_t q_prologue, int32_t policy, int32_t* tiles) {
  if (!tiles || n_rows <= 0 || T <= 0 || r_dim <= 0 || c_dim <= 0 || ntaps < 1 || ntaps > 8 || policy < POL_AUTO ||
      policy > POL_K1_2PCU) {
    set_error("vqx_wgrad_tiles: bad arguments");
    return -1;
  }
  const bool bf16 = dtype == VQX_BF16;
  const int bkv = bf16 ? 64 : 32;
  const bool gen = (T % bkv) != 0 || (n_rows % bkv) != 0;
  const int tm = (r_dim + 127) / 128;
  if (!gen && wgrad_tr_ok(n_rows, T, c_dim, ntaps, pad, dil > 0 ? dil : 1, bf16, q_prologue, policy))
    *tiles = tm * (c_dim / 64);
  else *tiles = tm * ((ntaps * c_dim + kBN - 1) / kBN);
  return 0;
}

extern "C" int vqx_wgrad_fixup_ok(int64_t n_rows, int32_t T, int32_t r_dim, int32_t c_dim, int32_t ntaps, int32_t pad,
                                  int32_t dil, int32_t dtype, int32_t slab_dtype, int32_t q_prologue, int32_t policy,
                                  int32_t* ok) {
  if (!ok || n_rows <= 0 || T <= 0 || r_dim <= 0 || c_dim <= 0 || ntaps < 1 || ntaps > 8) {
    set_error("vqx_wgrad_fixup_ok: bad arguments");
    return -1;
  }
  const bool bf16 = dtype == VQX_BF16;
  const bool gen = (T % 64) != 0 || (n_rows % 64) != 0;
  *ok = (bf16 && slab_dtype == VQX_BF16 && !gen &&
         wgrad_tr_ok(n_rows, T, c_dim, ntaps, pad, dil > 0 ? dil : 1, bf16, q_prologue, policy)) ? 1 : 0;
  return 0;
}

extern "C" int vqx_probe_enable(int32_t on) {
  g_probe_on = on != 0;  // pause / resume; the log is kept
  return 0;
}

extern "C" int vqx_probe_select(const int32_t* info5) {
  g_probe_sel_on = info5 != nullptr;
  if (info5)
    for (int i = 0; i < 5; ++i) g_probe_sel[i] = info5[i];
  return 0;
}

extern "C" int vqx_probe_clear(void) {
  g_probe.clear();
  g_probe_used = 0;
  return 0;
}

extern "C" int vqx_probe_count(int64_t* n) {
  if (!n) { set_error("vqx_probe_count: null"); return -1; }
  *n = (int64_t)g_probe.size();
  return 0;
}

extern "C" int vqx_probe_read(int64_t i, int32_t* info5, double* flops, float* ms) {
  if (i < 0 || i >= (int64_t)g_probe.size() || !info5 || !flops || !ms) { set_error("vqx_probe_read: bad index %lld", (long long)i); return -1; }
  const ProbeRec& r = g_probe[i];
  for (int k = 0; k < 5; ++k) info5[k] = r.info[k];
  *flops = r.flops;
  const hipError_t e = hipEventElapsedTime(ms, r.start, r.stop);
  if (e != hipSuccess) { set_error("vqx_probe_read: %s", hipGetErrorString(e)); return -1; }
  return 0;
}
