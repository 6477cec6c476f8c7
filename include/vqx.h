/*
 * vqx.h — C ABI of libvqx.so, the MI355X (gfx950) kernels behind the
 * vae_npvc VQ-VAE training step.
 *
 * The reference (Sinica-SLAM/vae_npvc) has no native layer: every op on its
 * hot path is a stock PyTorch call.  Each entry point below replaces one of
 * those calls (or a fused group of them); the reference site is cited per
 * function.  Paths are relative to the reference repository root.
 *
 * Conventions (all entry points):
 *   - every pointer is a DEVICE pointer owned by the caller (PyTorch's caching
 *     allocator in the Python host layer); nothing here allocates or frees;
 *   - calls are stream-ordered on `stream` (a hipStream_t, NULL = legacy
 *     stream) and never synchronise the host, so they can be captured into a
 *     hipGraph;
 *   - activations are "frame-major": row n = b*T + t, channels contiguous
 *     (the reference's (B, C, T) tensors transposed to (B*T, C));
 *   - return 0 on success, <0 on an invalid argument (-1) or a HIP launch
 *     error (-2); vqx_last_error() then holds thread-local text.
 */
#ifndef VQX_H
#define VQX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* vqx_stream_t; /* hipStream_t */

/* element types of activation / weight operands */
enum { VQX_F32 = 0, VQX_BF16 = 1 };

/* operand prologues, applied elementwise while a tile is staged into LDS */
enum {
  VQX_PRO_NONE = 0,
  VQX_PRO_LRELU = 1,      /* LeakyReLU(0.2)   layers.py:152, vqvae.py:171   */
  VQX_PRO_RELU = 2,       /* ReLU             vqvae.py:283,285              */
  VQX_PRO_SCALE_RELU = 3  /* ReLU(pro_scale*x) vqvae.py:316-317            */
};

/* epilogue flags of vqx_conv1d_fwd / vqx_conv1d_dgrad, applied in this order */
enum {
  VQX_EPI_BIAS = 1 << 0,    /* v += bias[c]                                    */
  VQX_EPI_ROWBIAS = 1 << 1, /* v += rowbias[(n/T)*cout + c]  (conv_cond term)  */
  VQX_EPI_MASK = 1 << 2,    /* v *= (mask[n][c] > 0 ? 1 : mask_slope)*mask_scale */
  VQX_EPI_RES = 1 << 3,     /* v += res[n][c]                                  */
  VQX_EPI_GNADD = 1 << 4,   /* v += (gn_h[n][c]-mean[b])*rstd[b]*gamma[c]+beta[c] */
  VQX_EPI_SPLIT = 1 << 5,   /* cols >= split_col -> out2[n][c-split_col] (f32,
                               '+=' when out2_accumulate)                      */
  VQX_EPI_OUTF32 = 1 << 6,  /* y stored as f32 instead of `dtype`              */
  VQX_EPI_ACT = 1 << 7,     /* y = act(v), act = epi_act (VQX_PRO_LRELU/RELU)  */
  VQX_EPI_ACT2 = 1 << 8,    /* also y2[n][c] = act(v) (dtype): the producer writes
                               the pre-activated copy its consumers read, so no
                               GEMM applies an activation while staging        */
  VQX_EPI_COLSUM = 1 << 9,  /* colsum_part[tile][c] = sum over the 128-frame row
                               tile of the stored fp32 value (before rounding):
                               the bias gradient of the layer y feeds, reduced
                               later by a VQX_WN_COLREDUCE table entry          */
  VQX_EPI_GNSTATS = 1 << 10, /* y is a GroupNorm input: stat_part[g128][tn][4] =
                               (count, mean, M2, 0) of the stored fp32 values of
                               each 128-frame x 128-channel tile; combined by
                               vqx_gn_finalize_tiles.  Needs T % 128 == 0 and
                               cout/gn_groups % 128 == 0                        */
  VQX_EPI_GNBWD = 1 << 11   /* y is the gradient dy of a GroupNorm output (GLU-
                               gated when gn_glu): stat_part[g128][tn][4] = per
                               tile (sum g*dh, sum g*dh*xhat) for group a (and b)
                               with u = gn_h [N][ldgn], the forward mean/rstd,
                               gamma, beta; consumed by vqx_gn_bwd(nparts > 0)  */
};
#define VQX_CONV_TILE_ROWS 128   /* frames per GEMM row tile (COLSUM partial rows) */

/*
 * Stride-1 Conv1d / ConvTranspose1d as an implicit-im2col GEMM on MFMA.
 *   fwd  : y[n][co] = epi( sum_{j,ci} w[co][j*cin+ci] * pro(x[n+j*dil-pad][ci]) )
 *          rows n+j*dil-pad outside the utterance of n read as zero (padding).
 *   dgrad: the same args with x = dy [N][cin], w = the FORWARD layer's packed
 *          weight [cout][ntaps*cin_fwd]; computes
 *          dx[n][ci] = epi( sum_{j,c} w[c][(ntaps-1-j)*cout_total.. ] ... )
 *          i.e. the transposed, tap-flipped conv; here `cin` = channels of dy
 *          (the forward layer's cout) and `cout` = the forward layer's cin.
 * Reference: nn.Conv1d / nn.ConvTranspose1d forward and autograd backward,
 * vqvae.py:156,174,257-265,286; layers.py:157,164,196,208,213.
 */
typedef struct vqx_conv_args {
  const void* x;             /* [N][ldx]                                       */
  const void* w;             /* packed weight [cout_fwd][ntaps*cin_fwd]        */
  void* y;                   /* [N][ldy]                                       */
  const float* bias;         /* [cout]                                         */
  const float* rowbias;      /* [B][cout]                                      */
  const void* res;           /* [N][ldres]  dtype                              */
  const void* mask;          /* [N][ldmask] dtype                              */
  const void* gn_h;          /* [N][ldgn]   dtype                              */
  const float* gn_mean_rstd; /* [B][2]                                         */
  const float* gn_gamma;     /* [cout]                                         */
  const float* gn_beta;      /* [cout]                                         */
  float* out2;               /* [N][ldo2] f32                                  */
  int64_t n_rows;            /* N = B*T                                        */
  int32_t T;                 /* frames per utterance                           */
  int32_t cin, cout, ntaps, pad;
  int32_t ldx, ldy, ldres, ldmask, ldgn, ldo2;
  int32_t dtype;             /* VQX_F32 | VQX_BF16                             */
  int32_t prologue;          /* VQX_PRO_*  (applied to x)                      */
  int32_t epilogue;          /* VQX_EPI_* flags                                */
  int32_t split_col, out2_accumulate;
  float pro_scale, mask_slope, mask_scale;
  void* y2;                  /* ACT2 destination [N][ldy2]                     */
  int32_t ldy2, epi_act;
  float* colsum_part;        /* COLSUM destination [ceil(N/128)][cout]         */
  float* stat_part;          /* GNSTATS / GNBWD destination [N/128][ceil(cout/128)][4] */
  int32_t gn_groups, gn_glu;
  /* GNADD with gn_stat_tiles != NULL: the GroupNorm statistics (G = 1) are
   * merged from the producing GEMM's GNSTATS tiles inside this launch (as
   * vqx_gn_finalize_tiles computes them, eps gn_eps) and written to
   * gn_mean_rstd [B][2]; needs T % 128 == 0 and cout % 128 == 0. */
  const float* gn_stat_tiles;
  float gn_eps;
  int32_t dil;               /* tap spacing (dilation, vqvae.py:166,274); 0 or 1 = dense.
                                Taps sit at n + j*dil - pad; 1 <= ntaps <= 8 and
                                0 <= pad <= (ntaps-1)*dil.  DGRAD takes the forward
                                layer's ntaps/dil and pad' = (ntaps-1)*dil - pad    */
  int32_t kernel_policy;     /* VQX_POLICY_* (ABI 122): which bf16 GEMM kernels this call may
                                use; 0 = automatic.  Per call, no process-wide state.         */
} vqx_conv_args;

/* Kernel policy of a conv GEMM call (vqx_conv_args / vqx_wgrad_args
 * .kernel_policy; the data-gradient args decide for vqx_conv1d_dgrad_wgrad):
 * AUTO picks by shape (3-tap, pad-1 bf16 layers with T % 128 == 0 run the
 * tap-reuse kernels, the 512-frame tall kernel where it fills the GPU, 1x1
 * layers the implicit-im2col kernel, layer pairs the fused DGRAD + WGRAD
 * launches); IM2COL keeps every GEMM on the implicit-im2col kernel and turns
 * the fused launches off; TALL256 / TALL512 force the tall tap-reuse kernel's
 * 256 / 512-frame tiles where they apply; TR128 keeps 3-tap layers on the
 * 128-frame tap-reuse kernel.  All produce the same values (tests compare
 * them); the choice is speed only. */
#define VQX_POLICY_AUTO 0
#define VQX_POLICY_IM2COL 1
#define VQX_POLICY_TALL256 2
#define VQX_POLICY_TALL512 3
#define VQX_POLICY_TR128 4
#define VQX_POLICY_K1_2PCU 5  /* ABI 125: as AUTO, but the bf16 1x1 FWD and DGRAD+WGRAD on the
                                 two-workgroups-per-CU kernels (AUTO: three per CU, one round
                                 with spare slots, since round 5) */

int vqx_conv1d_fwd(const vqx_conv_args* a, vqx_stream_t stream);
int vqx_conv1d_dgrad(const vqx_conv_args* a, vqx_stream_t stream);

/*
 * Weight gradient of a stride-1 conv as split-K partial slabs:
 *   slabs[s][r][j*c_dim + c] = sum_{n in split s} p[n][r] * pro(q[n + sign*(j*dil-pad)][c])
 * Conv1d  (dW[co][ci][j]): p = dy, q = x,  sign = +1.
 * ConvT1d (dW[ci][co][k-1-j]): p = x, q = du, sign = -1.
 * vqx_weight_norm_bwd reduces the slabs.  Reference: autograd of the convs
 * above (convolution_backward, 49% of the reference CPU step).
 */
typedef struct vqx_wgrad_args {
  const void* p;
  const void* q;
  void* slabs;       /* [splits][r_dim][ntaps*c_dim] of slab_dtype */
  int64_t n_rows;
  int32_t T, r_dim, c_dim, ntaps, pad, shift_sign, ldp, ldq;
  int32_t dtype, q_prologue, splits;
  float pro_scale;
  int32_t dil;       /* taps at n + sign*(j*dil - pad); 0 or 1 = dense */
  int32_t slab_dtype; /* VQX_F32, or VQX_BF16 (bf16 operands only): each split's fp32 partial
                         rounded once to bf16, half the slab bytes written here and read by
                         vqx_weight_norm_bwd, which sums them in fp32 */
  int32_t kernel_policy; /* VQX_POLICY_* (ABI 122); IM2COL: no tap-reuse weight-gradient kernel */
  /* In-launch ordered split-K reduction (ABI 127, optional: NULL = off).  With
   * fixup_dw set, the split that finishes an output tile last (one agent-scope
   * counter per tile) sums every split's slab of that tile in split order
   * 0, 1, ... in fp32 -- the order vqx_weight_norm_bwd sums slabs -- and
   * stores the fp32 weight gradient fixup_dw [r_dim][ntaps*c_dim]; a
   * weight-norm backward table entry then reads it as one fp32 "slab"
   * (splits 1), bit for bit the gradient it would have formed from the
   * slabs.  The slabs are still written (write-through, for the last split to
   * read).  fixup_counters: vqx_wgrad_tiles(...) uint32 counters, zero before
   * the first call and left zero by every call.  Needs the 3-tap tap-reuse
   * weight-gradient kernel and bf16 slabs (vqx_wgrad_fixup_ok). */
  float* fixup_dw;
  uint32_t* fixup_counters;
} vqx_wgrad_args;

int vqx_conv1d_wgrad(const vqx_wgrad_args* a, vqx_stream_t stream);
/* *ok = 1 when a weight gradient of this shape takes the in-launch split-K
 * reduction (fixup_dw), else 0 (ABI 127). */
int vqx_wgrad_fixup_ok(int64_t n_rows, int32_t T, int32_t r_dim, int32_t c_dim, int32_t ntaps, int32_t pad, int32_t dil,
                       int32_t dtype, int32_t slab_dtype, int32_t q_prologue, int32_t policy, int32_t* ok);

/*
 * One layer's data gradient (d, as vqx_conv1d_dgrad) and weight gradient (w,
 * as vqx_conv1d_wgrad) from the same output gradient, in one launch whose
 * workgroups interleave the two GEMMs (each CU runs one of each, so the data
 * gradient's fused epilogue overlaps the weight gradient's main loop) where a
 * fused instance covers the pair: bf16, no prologue, the 3-tap tap-reuse
 * kernels, and 1x1 layers (their data gradient's workgroups first, then the
 * weight gradient's in the slots they free).  Otherwise the two are launched in sequence
 * (weight gradient first).  *fused (may be NULL) = 1 for one launch, 0 for
 * two.  Results equal the separate calls bit for bit.  Replaces the two
 * autograd calls of one conv in the reference backward.
 */
int vqx_conv1d_dgrad_wgrad(const vqx_conv_args* d, const vqx_wgrad_args* w, int32_t* fused, vqx_stream_t stream);

/*
 * Weight norm (torch.nn.utils.weight_norm, dim=0; applied at vqvae.py:203-208,
 * 329-334): w = g * v / ||v|| per row o of v[rows][cols] (Conv1d rows = cout,
 * ConvT rows = cin).  The forward packs w into the effective-conv layout the
 * GEMMs read: w_packed[co][j*cin + ci] in `dtype`.
 * kind 0: Conv1d v[cout][cin][k]; kind 1: ConvTranspose1d v[cin][cout][k]
 * (effective tap j' = k-1-j).  Descriptors are batched: one launch packs
 * every layer of the model.
 */
#define VQX_WN_COLREDUCE 2  /* table entry kind: dv[c] = sum_{r < cin} v[r*cout + c] (bias /
                               GroupNorm-affine gradients from per-tile or per-utterance
                               partials, reduced in the same backward launch)        */
/* Resampling convs of the multi-resolution models (vqvae.py:144-156 /
 * 243-263, vqvae2.py:197-226 / 297-319): kernel k = 2s, stride s, padding
 * p = s/2 + s%2 (ConvT output_padding s%2).  With frames folded s at a time
 * (x'[u] = x[s*u .. s*u+s-1], a reinterpretation of the frame-major [N][C]
 * layout as [N/s][s*C]) the strided conv is a stride-1, 3-tap, pad-1 conv:
 *   w_packed[r][m][q*C + c] = w[r][c][s*(m-1) + q + p]  (0 when outside [0,k))
 * for rows r (kind 3: cout of v[cout][cin][k], C = cin; kind 4: cin of the
 * ConvT's v[cin][cout][k], C = cout), m in 0..2, q in 0..s-1.  The strided
 * Conv1d runs as vqx_conv1d_fwd on the folded input; the ConvTranspose1d
 * (its adjoint) as vqx_conv1d_dgrad; both gradients follow the same way and
 * the backward folds the 3-tap wgrad slabs [splits][r][3*s*C] back to v. */
#define VQX_WN_RESAMPLE 3    /* strided Conv1d, v[cout][cin][k]          */
#define VQX_WN_RESAMPLE_T 4  /* strided ConvTranspose1d, v[cin][cout][k] */
typedef struct vqx_wn_layer {
  const float* v;       /* [rows][cols] */
  const float* g;       /* [rows]       */
  void* w_packed;       /* [cout][k*cin] dtype */
  float* norm;          /* [rows] ||v_o|| saved for the backward */
  float* dv;            /* bwd: [rows][cols] */
  float* dg;            /* bwd: [rows] */
  const void* slabs;    /* bwd: wgrad slabs (slab_dtype) */
  int32_t kind, cout, cin, k, splits, dtype;
  int32_t stride, pad;  /* kinds VQX_WN_RESAMPLE(_T) only */
  int32_t slab_dtype;   /* VQX_F32 | VQX_BF16 (vqx_wgrad_args.slab_dtype) */
} vqx_wn_layer;

/* `layers_host` sizes the launch; the kernels read the same table from the
 * device copy `layers_dev` (built once by the caller, so a captured graph
 * replays without host work). */
int vqx_weight_norm_fwd(const vqx_wn_layer* layers_host, const vqx_wn_layer* layers_dev,
                        int32_t n_layers, vqx_stream_t stream);
/* The same with flags (ABI 125): VQX_WNF_NORMS_READY skips the ConvTranspose
 * row norms (kind 1): vqx_adam_step_wn has written them for the current v. */
#define VQX_WNF_NORMS_READY 1
int vqx_weight_norm_fwd_flags(const vqx_wn_layer* layers_host, const vqx_wn_layer* layers_dev,
                              int32_t n_layers, int32_t flags, vqx_stream_t stream);
int vqx_weight_norm_bwd(const vqx_wn_layer* layers_host, const vqx_wn_layer* layers_dev,
                        int32_t n_layers, vqx_stream_t stream);
/* The same launch, also leaving the sum of squares of every gradient value it
 * writes (dv, dg, column reductions) as per-wave partials in
 * sq_partials[0 .. count) (ABI 125; count from vqx_weight_norm_bwd_partials):
 * the global gradient norm of clip_grad_norm_ (trainer/basic.py:63-67)
 * without re-reading the 125 MB gradient.  vqx_sq_norm_finish then sums the
 * partials and g^2 over the flat ranges [off, off+len) the weight-norm
 * backward does not write (ranges: int64 pairs, device memory), each in a
 * fixed order, into out[0] -- what vqx_grad_sq_norm computes, summed in
 * another order. */
int vqx_weight_norm_bwd_partials(const vqx_wn_layer* layers_host, int32_t n_layers, int64_t* count);
int vqx_weight_norm_bwd_sq(const vqx_wn_layer* layers_host, const vqx_wn_layer* layers_dev,
                           int32_t n_layers, float* sq_partials, int64_t sq_capacity, vqx_stream_t stream);
int vqx_sq_norm_finish(const float* partials, int64_t n_partials, const float* g, const int64_t* ranges,
                       int32_t n_ranges, float* scratch /* >= 256 floats */, float* out, vqx_stream_t stream);
/* vqx_sq_norm_finish followed by vqx_adam_hyper (same arguments, same
 * results) with the second folded into the finish's last launch (ABI 126). */
int vqx_sq_norm_finish_adam(const float* partials, int64_t n_partials, const float* g, const int64_t* ranges,
                            int32_t n_ranges, float* scratch, float* out, int64_t* step, double lr0, double gamma,
                            int32_t step_size, double beta1, double beta2, double eps, float* hyper,
                            vqx_stream_t stream);

/*
 * GroupNorm statistics (nn.GroupNorm, layers.py:154 (G=1), layers.py:201
 * (G=2); eps 1e-5): mean and 1/sqrt(var+eps) over (C/G, T) per utterance.
 * x [N][ldx] dtype, C channels; out mean_rstd[B][G][2] f32.  Two-pass
 * (mean, then centred sum of squares) per (b, g).
 */
int vqx_groupnorm_stats(const void* x, int32_t ldx, int32_t dtype, int64_t n_rows, int32_t T,
                        int32_t C, int32_t G, float eps, float* partials /* >= B*G*24 */,
                        float* mean_rstd, vqx_stream_t stream);

/*
 * Fused GroupNorm(G=2) + gated tanh/sigmoid unit, decoder ResSkip block
 * (layers.py:236-242):  g[n][c] = tanh(h(n,c)) * sigmoid(h(n,c+C/2)),
 * h = (u - mean)*rstd*gamma + beta.  u [N][ldu], g [N][ldg], C = 2*half.
 */
int vqx_gn_glu_fwd(const void* u, int32_t ldu, void* g, int32_t ldg, int32_t dtype, int64_t n_rows,
                   int32_t T, int32_t C, const float* mean_rstd, const float* gamma, const float* beta,
                   vqx_stream_t stream);

/* vqx_gn_glu_fwd with the GroupNorm statistics merged from the producing
 * GEMM's GNSTATS tiles (G = 2, as vqx_gn_finalize_tiles computes them) inside
 * the same launch; mean_rstd [B][2][2] is written for the backward.
 * Needs T % 128 == 0 and C % 256 == 0. */
int vqx_gn_glu_fwd_tiles(const void* u, int32_t ldu, void* g, int32_t ldg, int32_t dtype, int64_t n_rows,
                         int32_t T, int32_t C, const float* parts, float eps, float* mean_rstd,
                         const float* gamma, const float* beta, vqx_stream_t stream);

/* GroupNorm(G=1) + LeakyReLU(0.2): g = lrelu((h - mean)*rstd*gamma + beta),
 * the operand of each further conv of a residual stack with stack_layers > 1
 * (layers.py:156-161).  h, g [N][ld*] dtype; mean_rstd [B][2] from
 * vqx_groupnorm_stats / vqx_gn_finalize_tiles.  The backward needs no kernel
 * of its own: the next conv's DGRAD applies the LeakyReLU derivative with
 * VQX_EPI_MASK (mask = g, slope 0.2) and vqx_gn_bwd(glu = 0) the GroupNorm. */
int vqx_gn_lrelu_fwd(const void* h, int32_t ldh, void* g, int32_t ldg, int32_t dtype, int64_t n_rows, int32_t T,
                     int32_t C, const float* mean_rstd, const float* gamma, const float* beta, vqx_stream_t stream);

/*
 * Backward of GroupNorm(G) optionally preceded by the gated unit:
 *   glu=1: dy is dL/dg [N][C/2], u is the GN input [N][C]: computes dL/dh
 *          through tanh*sigmoid, then through GroupNorm, into du [N][C].
 *   glu=0: dy is dL/d(GN output) [N][C].
 * Also accumulates per-utterance column sums of du (for the conv bias and
 * conv_cond gradients) into colsum[B][C] and dgamma/dbeta partials
 * [B][C] (summed over B by the caller's reduction).
 * Reference: autograd of layers.py:236-242 and 170-176.
 */
int vqx_gn_bwd(const void* dy, int32_t lddy, const void* u, int32_t ldu, void* du, int32_t lddu,
               int32_t dtype, int64_t n_rows, int32_t T, int32_t C, int32_t G, int32_t glu,
               const float* mean_rstd, const float* gamma, const float* beta,
               float* partials /* nparts == 0: workspace >= B*64*G */,
               int32_t nparts /* 0: reduce here; > 0: partials hold the producing GEMM's
                                 VQX_EPI_GNBWD tiles, nparts per utterance */,
               float* colsum_b /* [B][C] */, float* dgamma_b /* [B][C] */, float* dbeta_b /* [B][C] */,
               vqx_stream_t stream);

/* GroupNorm statistics from a GEMM's VQX_EPI_GNSTATS tiles (see there):
 * mean_rstd[B][G][2], combined per (utterance, group) in double. */
int vqx_gn_finalize_tiles(const float* parts, int64_t n_rows, int32_t T, int32_t C, int32_t G, float eps,
                          float* mean_rstd, vqx_stream_t stream);

/*
 * Sum over rows: out[c] (+)= sum_n x[n][c] (f32 accumulation, deterministic
 * two-level tree).  Used for conv bias gradients and for reducing [B][C]
 * partials.  accumulate=1 adds into out.
 */
int vqx_colsum(const void* x, int32_t ldx, int32_t dtype, int64_t n_rows, int32_t C,
               float* partials /* >= 64*C */, float* out, int32_t accumulate, vqx_stream_t stream);

/*
 * The first level of vqx_colsum alone (ABI 126): partials[p][c] = the sum of
 * row part p of column c, p < vqx_colsum_parts(n_rows, C, dtype) <= 64.  The
 * caller reduces them later, e.g. as a VQX_WN_COLREDUCE entry of the batched
 * weight-norm backward (a conv bias gradient without a launch of its own).
 */
int vqx_colsum_parts(int64_t n_rows, int32_t C, int32_t dtype, int32_t* nparts);
int vqx_colsum_partials(const void* x, int32_t ldx, int32_t dtype, int64_t n_rows, int32_t C,
                        float* partials /* >= nparts * C */, vqx_stream_t stream);

/*
 * Frame-major copy of the (B, C, T) input batch, with dtype conversion
 * (the reference's z.transpose(1,2).contiguous(), layers_vq.py:274-276).
 */
int vqx_nct_to_ntc(const float* x_nct, int32_t B, int32_t C, int32_t T, void* y, int32_t ldy,
                   int32_t dtype, vqx_stream_t stream);
int vqx_ntc_to_nct(const void* y, int32_t ldy, int32_t dtype, int32_t B, int32_t C, int32_t T,
                   float* x_nct, vqx_stream_t stream);

/*
 * log_loss (layers.py:283-296, reduction 'frame_mean') fused with its
 * gradient: loss = sum 0.5*(log2pi + (x - xhat)^2) / (B*T);
 * dxhat = (xhat - x) * grad_scale (grad_scale = dL/dloss / (B*T)).
 * x is the reference (B, C, T) f32 batch; xhat is frame-major f32.
 * loss_out[0] receives the loss (deterministic reduction).
 */
int vqx_logloss_fwd_bwd(const float* x_nct, const float* xhat, int32_t ldxh, int32_t B, int32_t C,
                        int32_t T, float grad_scale, void* dxhat, int32_t lddx, int32_t dtype,
                        float* loss_out, float* partials, vqx_stream_t stream);
/* The same, and in its final sum launch also extra_out[0] = the sum of
 * extra_partials[0 .. n_extra) in the order vqx_vq_forward sums its
 * commitment partials (ABI 126: the VQ kernel then runs with sqerr_out NULL,
 * one launch fewer). */
int vqx_logloss_fwd_bwd_x(const float* x, const float* xhat, int32_t ldxh, int32_t B, int32_t C, int32_t T,
                          float grad_scale, void* dxhat, int32_t lddx, int32_t dtype, float* loss_out,
                          float* partials, const float* extra_partials, int32_t n_extra, float* extra_out,
                          vqx_stream_t stream);
/* The same without the final sum launch (ABI 128): the per-workgroup
 * partials only, their count in *n_parts (at most 1024); the total is
 * (1/(B*T)) * their sum in the order vqx_logloss_fwd_bwd adds them
 * (vqx_vq_ema_update_close sums them so). */
int vqx_logloss_parts(const float* x, const float* xhat, int32_t ldxh, int32_t B, int32_t C, int32_t T,
                      float grad_scale, void* dxhat, int32_t lddx, int32_t dtype, float* partials, int32_t* n_parts,
                      vqx_stream_t stream);

/*
 * EMA vector-quantizer forward (EMAVectorQuantizer.forward,
 * layers_vq.py:268-323, distances :285-289, argmin :291, gather :292,
 * commitment loss :301,308-309; update_emb statistics :207-211):
 *   dist[n][k] = (||z_n||^2 + ||e_k||^2) - 2 z_n.e_k   (fp32 MFMA)
 *   idx[n]     = first argmin_k dist[n][k]               (int64)
 *   zq[n]      = E[idx[n]]  (f32 [N][D]) and zq_c (dtype, decoder input)
 *   sqerr      : sum_n ||zq_n - z_n||^2  into sqerr_out[0] (deterministic)
 *   bsum[k][d] += sum_{n: idx=k} z[n][d], bcnt[k] += |{n: idx=k}|
 *                 (deterministic: 512-frame chunks sorted by code, segmented
 *                 sums, chunk tables reduced in order; pass NULL to skip, e.g.
 *                 eval / encode())
 * z [N][D] f32 (frame-major, D = z_dim in {64, 128, 256}), E [K][D] f32,
 * K % 16 == 0, K <= 2048.  `partials` is a caller workspace of
 * >= vqx_vq_workspace(N, K, D, bsum != NULL) floats.
 */
int vqx_vq_forward(const float* z, int64_t n_rows, int32_t D, const float* E, int32_t K,
                   int64_t* idx, float* zq, void* zq_c, int32_t zq_c_dtype, float* sqerr_out,
                   float* partials, float* bsum, float* bcnt, vqx_stream_t stream);
/* Workspace (floats) vqx_vq_forward needs for N frames and K codes of width
 * D, with or without the EMA statistics (ABI 123: D added). */
int vqx_vq_workspace(int64_t n_rows, int32_t K, int32_t D, int32_t with_stats, int64_t* floats);
/* The EMA statistics part of vqx_vq_forward on its own (bsum = one-hot^T z,
 * bcnt = counts of idx; update_emb's onehot matmul, layers_vq.py:207-211),
 * for callers that run it on another stream than the distance kernel.
 * `partials` is the same workspace (with stats); it does not touch the
 * commitment partials, so it may run beside vqx_vq_forward's sqerr sum. */
int vqx_vq_stats(const float* z, int64_t n_rows, int32_t D, const int64_t* idx, int32_t K, float* partials,
                 float* bsum, float* bcnt, vqx_stream_t stream);

/*
 * EMA codebook update (update_emb, layers_vq.py:203-233; init_emb :192-201):
 *   emb_sum  = mu*emb_sum  + (1-mu)*bsum;  emb_elem = mu*emb_elem + (1-mu)*bcnt
 *   usage    = emb_elem >= threshold
 *   E        = usage ? emb_sum/emb_elem : rand_rows
 *   diag[0..3] = {entropy (perplexity of bcnt), used_curr, usage, diff_emb}
 * rand_rows [K][D] are the rows z[perm[:K]] gathered by vqx_gather_rows.
 * partials: workspace of ceil(K*D/1024) + 1 words, the last a counter that
 * must be zero before the first call (each call leaves it zero; ABI 128: one
 * launch, its last workgroup runs the per-code pass).  Deterministic (fixed
 * summation order).
 */
int vqx_vq_ema_update(float* emb_sum, float* emb_elem, float* E, const float* bsum,
                      const float* bcnt, const float* rand_rows, int32_t K, int32_t D, float mu,
                      float threshold, float* diag, float* partials, vqx_stream_t stream);
/* The same, and bsum / bcnt are zero afterwards (ABI 126): the next step's
 * vqx_vq_forward accumulates into them without a zero-fill launch. */
int vqx_vq_ema_update_clear(float* emb_sum, float* emb_elem, float* E, float* bsum, float* bcnt,
                            const float* rand_rows, int32_t K, int32_t D, float mu, float threshold, float* diag,
                            float* partials, vqx_stream_t stream);
/* vqx_vq_ema_update_clear that also closes the training step's forward in
 * its last workgroup (ABI 128), the work of two one-workgroup launches:
 *   out[i][0] = scale[i] * (parts[i][0] + ... + parts[i][n[i]-1]), i < 2
 *     (parts[i] NULL: none), summed in the order of vqx_logloss_fwd_bwd_x's
 *     final launch (the log-loss total from vqx_logloss_parts' partials with
 *     scale 1/(B*T); the commitment sum from vqx_vq_forward's partials);
 *   then, with pub_box != NULL, pub_src[0 .. pub_n) published into mailbox
 *     slot pub_slot with number pub_seq as vqx_mailbox_publish does, after
 *     the sums and diag are stored (pub_src may hold them);
 *   with rows_src != NULL, the dead-code rows read straight from it: row k of
 *     rand_rows is rows_src[rows_host[k] * rows_ld ..] (a zero row for a
 *     negative index; rows_host: n_rows == K <= 512 host int32 indices, copied
 *     into the launch's arguments; rand_rows is then not read and may be
 *     NULL): vqx_gather_rows_host folded in.
 * The values equal those of the separate launches bit for bit. */
typedef struct {
  const float* parts[2];
  int32_t n[2];
  float scale[2];
  float* out[2];
  const float* pub_src;
  int32_t pub_n;
  float* pub_copy;     /* device copy of the published values, or NULL */
  void* pub_box;       /* vqx_mailbox_create's device pointer, or NULL */
  int32_t pub_slot, pub_slots, pub_floats;
  uint32_t pub_seq;
  const float* rows_src;   /* z, or NULL: rand_rows as given */
  int32_t rows_ld, n_rows;
  const int32_t* rows_host;
} vqx_step_close;
int vqx_vq_ema_update_close(float* emb_sum, float* emb_elem, float* E, float* bsum, float* bcnt,
                            const float* rand_rows, int32_t K, int32_t D, float mu, float threshold, float* diag,
                            float* partials, const vqx_step_close* close, vqx_stream_t stream);

/* out[i][:] = src[rows[i]][:] for i < n_out  (f32, row length D).  rows are
 * int64 indices; negative indices write zero rows (rows owned by another
 * rank in data-parallel training). */
int vqx_gather_rows(const float* src, int32_t ld_src, const int64_t* rows, int32_t n_out,
                    int32_t D, float* out, vqx_stream_t stream);

/* The same gather with the row indices in HOST memory (int32, read during
 * the call and passed to the kernels by value, 512 rows a launch): no
 * host-to-device copy on the stream.  Replaces the reference's
 * `_z[torch.randperm(N)][:K]` indexing with a CPU permutation
 * (layers_vq.py:197,213), whose index tensor torch copies to the device. */
int vqx_gather_rows_host(const float* src, int32_t ld_src, const int32_t* rows, int32_t n_out,
                         int32_t D, float* out, vqx_stream_t stream);

/* Commitment-loss gradient (layers_vq.py:301 backward):
 *   dz[n][d] = scale * (z[n][d] - zq[n][d])  written in dtype. */
int vqx_vq_commit_bwd(const float* z, const float* zq, int64_t count, float scale, void* dz,
                      int32_t dtype, vqx_stream_t stream);
/* The same over [n_rows][D] rows, plus the column sums of the dz it stores
 * (ABI 126): partials[p][d] = sum of dz[n][d] over the rows n of part p (rows
 * n_rows*p/P .. n_rows*(p+1)/P, P = VQX_COMMIT_PARTS; empty parts write 0),
 * the first level of the bias gradient of the conv producing z.  D % 4 == 0,
 * D <= 1024. */
#define VQX_COMMIT_PARTS 256
int vqx_vq_commit_bwd_cs(const float* z, const float* zq, int64_t n_rows, int32_t D, float scale, void* dz,
                         int32_t dtype, float* partials /* [VQX_COMMIT_PARTS][D] */, vqx_stream_t stream);

/* Jitter (layers_vq.py:353-379): y[b][t][:] = x[b][src_t[t]][:]. */
int vqx_time_gather(const void* x, void* y, int32_t B, int32_t T, int32_t C, const int32_t* src_t,
                    int32_t dtype, vqx_stream_t stream);

/* Speaker embedding lookup (layers.py:42-54, nn.Embedding) and its
 * backward scatter-add (dense weight gradient). */
int vqx_embedding_fwd(const float* weight, const int64_t* ids, int32_t B, int32_t D, float* out,
                      vqx_stream_t stream);
int vqx_embedding_bwd(const float* dout, const int64_t* ids, int32_t B, int32_t D, float* dweight,
                      vqx_stream_t stream);
/* The dense weight gradient in one pass (ABI 126): every row r < n_rows of
 * dweight is written, dweight[r] (+)= sum over b with ids[b] == r of dout[b]
 * in batch order (0 for ids absent from the batch; accumulate = 1 adds).  No
 * zero-fill launch before it.  Any B (round 6): ids are staged 1024 at a
 * time, each chunk's sum added to the row in chunk order. */
int vqx_embedding_bwd_rows(const float* dout, const int64_t* ids, int32_t B, int32_t D, int32_t n_rows,
                           float* dweight, int32_t accumulate, vqx_stream_t stream);

/* Small dense GEMM for the time-constant conv_cond term (vqvae.py:309-312):
 * out[b][o] = sum_i W[o][i] * c[b][i] + bias[o]   (f32, W from weight norm
 * in f32).  And its backward:  dW[o][i] += sum_b dout[b][o] * c[b][i],
 * dc[b][i] += sum_o dout[b][o] * W[o][i]. */
/* All ResSkip blocks' speaker-conditioning linears in one launch (conv_cond on
 * the time-constant embedding, layers.py:218-236; table on the device).
 * fwd: out_l[b][o] = W_l[o][:] . c[b][:] + bias_l[o].
 * bwd: dW_l = dout_l^T c, dbias_l = colsum(dout_l) (both overwritten) and
 *      dc[b][i] = sum_l sum_o dout_l[b][o] W_l[o][i] (overwritten; NULL skips),
 *      reduced deterministically from split-K partials
 *      [n * ceil(O/64)][B][I] f32 (caller workspace). */
typedef struct vqx_linear_layer {
  const float* W;      /* [O][I] */
  const float* bias;   /* [O] or NULL */
  float* out;          /* fwd [B][O] */
  const float* dout;   /* bwd [B][O] */
  float* dW;           /* bwd [O][I] */
  float* dbias;        /* bwd [O] or NULL */
} vqx_linear_layer;
int vqx_linear_batched_fwd(const vqx_linear_layer* table_dev, int32_t n, const float* c, int32_t B,
                           int32_t I, int32_t O, vqx_stream_t stream);
int vqx_linear_batched_bwd(const vqx_linear_layer* table_dev, int32_t n, const float* c, int32_t B,
                           int32_t I, int32_t O, float* dc, float* partials, vqx_stream_t stream);
/* The same with c[b] = emb[ids[b]] (ABI 126): the embedding lookup
 * (vqx_embedding_fwd) folded into the operand loads, for I = 128, B <= 64,
 * O % 64 == 0 and a 16-B aligned table (anything else: an error). */
int vqx_linear_batched_fwd_ids(const vqx_linear_layer* table_dev, int32_t n, const float* emb,
                               const int64_t* ids, int32_t B, int32_t I, int32_t O, vqx_stream_t stream);
/* The training step's prologue as one launch (ABI 128): the three
 * independent jobs a step begins with --
 *   vqx_linear_batched_fwd_ids(cond_table_dev, n_cond, emb, ids, B, I, O)
 *     (the speaker conditioning, vqvae.py decoder inputs),
 *   vqx_nct_to_ntc(x_nct, xB, C, T, y, ldy, y_dtype) (the input's layout) and
 *   vqx_weight_norm_fwd_flags(wn_host, wn_dev, n_wn, VQX_WNF_NORMS_READY)
 *     (the ConvTranspose packs; their row norms must be current) --
 * with the three calls' results bit for bit, in one grid.  A job is skipped
 * with n_cond = 0, x_nct = NULL or n_wn = 0; n_wn <= 256; the conditioning
 * job has vqx_linear_batched_fwd_ids's limits (anything else: an error). */
int vqx_step_prologue(const vqx_wn_layer* wn_host, const vqx_wn_layer* wn_dev, int32_t n_wn,
                      const vqx_linear_layer* cond_table_dev, int32_t n_cond, const float* emb,
                      const int64_t* ids, int32_t B, int32_t I, int32_t O, const float* x_nct, int32_t xB,
                      int32_t C, int32_t T, void* y, int32_t ldy, int32_t y_dtype, vqx_stream_t stream);
int vqx_linear_batched_bwd_ids(const vqx_linear_layer* table_dev, int32_t n, const float* emb,
                               const int64_t* ids, int32_t B, int32_t I, int32_t O, float* dc, float* partials,
                               vqx_stream_t stream);

int vqx_linear_f32(const float* c, const float* W, const float* bias, int32_t B, int32_t I,
                   int32_t O, float* out, vqx_stream_t stream);
int vqx_linear_bwd_f32(const float* dout, const float* c, const float* W, int32_t B, int32_t I,
                       int32_t O, float* dW, float* dc, vqx_stream_t stream);

/*
 * Global gradient norm + fused Adam (trainer/basic.py:63-69:
 * clip_grad_norm_(max_norm) then torch.optim.Adam(betas, eps, wd=0)).
 * grad_sq_norm: out[0] = sum g^2 over the flat buffer (deterministic;
 *   partials >= 1024 floats).
 * adam_hyper: increments the device step counter t and writes
 *   hyper[8] = {lr_t, lr_t/(1-b1^t), sqrt(1-b2^t), t, 1-b1, b2, 1-b2, eps}
 *   with every scalar formed in double like torch's Python-float math, then
 *   rounded to f32; lr_t = lr0*gamma^floor((t-1)/step_size) (StepLR,
 *   basic.py:43-46, stepped once per iteration).  Graph-capturable.
 * adam_step: coef = min(1, max_norm/(sqrt(sumsq)+1e-6)) when max_norm > 0;
 *   g' = g*coef; m = lerp(m, g', 1-b1); v = v*b2 + ((1-b2)*g')*g';
 *   p += -(lr/bc1) * (m / (sqrt(v)/sqrt(bc2) + eps))   (torch single-tensor
 *   Adam operation order).
 */
int vqx_grad_sq_norm(const float* g, int64_t n, float* partials, float* out, vqx_stream_t stream);
int vqx_adam_hyper(int64_t* step, double lr0, double gamma, int32_t step_size, double beta1,
                   double beta2, double eps, float* hyper, vqx_stream_t stream);
int vqx_adam_step(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper,
                  const float* sumsq, float max_norm, vqx_stream_t stream);
/* adam_step with the next forward's weight-norm preparation fused in (ABI
 * 125; replaces the per-step torch weight_norm recomputation of
 * w = g*v/||v||, vqvae.py:203-208 / 329-334, that vqx_weight_norm_fwd does
 * otherwise).  rows: weight-normed convs (vqx_wn_layer with v, g pointing into
 * p; kind 0 needs w_packed) whose rows of v and gains g this launch updates,
 * writing norm[o] = ||v_o|| of the updated row and, for kind 0, the packed
 * weights -- bit for bit what vqx_weight_norm_fwd computes from the updated
 * parameters; kind 1 (ConvT) rows get their norms, to be packed by
 * vqx_weight_norm_fwd_flags(VQX_WNF_NORMS_READY).  segs: (offset, length)
 * int64 pairs covering every other element of p (host and device copies);
 * rows + segs must cover [0, n) exactly: the host rejects overlapping ranges
 * (round 6) and p, g, m, v that are not 16-B aligned.  The update of every
 * element is adam_step's, bit for bit.  At most 128 layers and 128 segments. */
int vqx_adam_step_wn(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper,
                     const float* sumsq, float max_norm, const vqx_wn_layer* rows_host,
                     const vqx_wn_layer* rows_dev, int32_t n_layers, const int64_t* segs_host,
                     const int64_t* segs_dev, int32_t n_segs, vqx_stream_t stream);

/* RAdam, optim_type: RAdam (replaces trainer/radam.py:5-78 RAdam.step, built
 * by trainer/basic.py:30-34 with betas (0.5, 0.999), weight_decay 0).
 * radam_hyper: increments t and writes hyper[9] = {lr_t, -ss*lr_t, rect, t,
 *   b1, 1-b1, b2, 1-b2, eps}: N_max = 2/(1-b2)-1, N = N_max - 2t b2^t/(1-b2^t);
 *   rect = N >= 5; ss = sqrt((1-b2^t)(N-4)/(N_max-4)(N-2)/N N_max/(N_max-2))
 *   / (1-b1^t) when rect, else 1/(1-b1^t) (radam.py:49-59), all in double
 *   like the Python floats, then rounded to f32; lr_t as adam_hyper (StepLR).
 * radam_step: g' = coef*g (clip as adam_step); v = v*b2 + ((1-b2)*g')*g';
 *   m = m*b1 + (1-b1)*g'; p += (-ss*lr) * (m / (sqrt(v) + eps)) when rect,
 *   else p += (-ss*lr) * m (radam.py:41-42, 64-71). */
int vqx_radam_hyper(int64_t* step, double lr0, double gamma, int32_t step_size, double beta1,
                    double beta2, double eps, float* hyper, vqx_stream_t stream);
int vqx_radam_step(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper,
                   const float* sumsq, float max_norm, vqx_stream_t stream);

/*
 * Straight-through VectorQuantizer (use_ema: false; layers_vq.py:9-163,
 * reduction 'frame_mean', target_norm 1.0, z_dim 64, 128 or 256).
 * vqx_vq_normalize (embed_norm: true): the codebook parameter E [K][D] is
 *   renormalised in place (embed_norm(), :28-33) and emb_norm = E/||E||
 *   (:99), e_len = ||E|| after that step; z_norm = z/||z|| (:97), z_len =
 *   ||z||; normloss_out = sum (z_norm - z)^2 (:125-126; partials >= N/4+1).
 *   Then vqx_vq_forward(z_norm, emb_norm, ..., bsum, bcnt) gives idx, z_q,
 *   the commitment sum and the per-code sums/counts the backward uses.
 * vqx_vq_perplexity: exp(-sum p log(p + 1e-10)), p = counts/N (:112-114).
 * vqx_vq_plain_bwd: gradients of x_loss + z_qut + beta*z_enc (scale =
 *   2/(B*T)): dz [N][D] (dtype) from the decoder's straight-through gradient
 *   dzq (zeroed on frames the Jitter replaced: src_t[t] != t; NULL = no
 *   jitter) plus the commitment / normalisation terms through z/||z||, and
 *   the codebook-parameter gradient dE [K][D] f32 (overwritten) through
 *   E/||E|| (or directly when normalize = 0, emb = E).
 */
int vqx_vq_normalize(const float* z, int64_t n_rows, int32_t D, float* E, int32_t K, float* z_norm,
                     float* z_len, float* emb_norm, float* e_len, float* partials, float* normloss_out,
                     vqx_stream_t stream);
int vqx_vq_perplexity(const float* counts, int32_t K, int64_t n_rows, float* out, vqx_stream_t stream);
int vqx_vq_plain_bwd(const float* z, const float* z_norm, const float* z_len, const float* zq,
                     const void* dzq, const int32_t* src_t, int32_t T, int64_t n_rows, int32_t D,
                     int32_t normalize, float beta, float scale, void* dz, int32_t dtype, const float* bsum,
                     const float* bcnt, const float* emb, const float* e_len, int32_t K, float* dE,
                     vqx_stream_t stream);

/* dst[r][c] = act(scale * src[r][c]) with dtype conversion (act = VQX_PRO_*;
 * the decoder's ReLU(sqrt(1/11) * skip) operand, vqvae.py:316-317). */
int vqx_scale_act_2d(const void* src, int32_t ld_src, int32_t src_dtype, void* dst, int32_t ld_dst,
                     int32_t dst_dtype, int64_t rows, int32_t cols, float scale, int32_t act,
                     vqx_stream_t stream);

/* 2-D strided copy with dtype conversion: dst[r][c] = src[r][c] for r < rows,
 * c < cols; src == NULL fills zeros.  Used for the decoder's skip-sum cast
 * and the residual/skip gradient buffers of the backward. */
int vqx_convert_2d(const void* src, int32_t ld_src, int32_t src_dtype, void* dst, int32_t ld_dst,
                   int32_t dst_dtype, int64_t rows, int32_t cols, vqx_stream_t stream);
/* convert_2d(src, dst) and, in the same launch, zero_dst[r][c] = 0 for r <
 * zero_rows, c < zero_cols (dst's dtype; ABI 126: the decoder backward's
 * dL/dskip copy and the zero dL/dx at the decoder output in one launch). */
int vqx_convert_2d_zero2(const void* src, int32_t ld_src, int32_t src_dtype, void* dst, int32_t ld_dst,
                         int32_t dst_dtype, int64_t rows, int32_t cols, void* zero_dst, int32_t ld_zero,
                         int64_t zero_rows, int32_t zero_cols, vqx_stream_t stream);

/* Work units per split of the weight-gradient kernel that vqx_conv1d_wgrad
 * would launch for these arguments, one unit = one 4-wave group (two per CU
 * fill the GPU): 3-tap, pad-1 bf16 layers with T % 64 == 0 and
 * c_dim % 64 == 0 run the tap-reuse kernel (128 rows x 3 taps x 64 channels
 * per tile, two 4-wave K groups per tile), the rest one group per 128 x 128
 * tile.  Callers size `splits` (and the slab buffer) from it. */
int vqx_wgrad_tiles(int64_t n_rows, int32_t T, int32_t r_dim, int32_t c_dim, int32_t ntaps, int32_t pad,
                    int32_t dil, int32_t dtype, int32_t q_prologue, int32_t kernel_policy /* ABI 125 */,
                    int32_t* tiles);

/* Thread-local description of the last failure. */
const char* vqx_last_error(void);

/* Launch probe (measurement only; its log and switches are per host thread,
 * so calls on other threads are unaffected).  While on,
 * each conv GEMM launch records a start/stop event pair stamped on its own
 * dispatch (hipExtLaunchKernelGGL); after the stream is synchronised,
 * vqx_probe_read returns per launch {dtype, mode, prologue, gen, epilogue kind},
 * the algorithmic FLOPs and the kernel duration in ms.  enable(0/1) pauses /
 * resumes recording (an event-stamped dispatch costs a few us of queue time,
 * so callers sample); clear() empties the log. */
int vqx_probe_enable(int32_t on);
/* Record only the launches whose {dtype, mode, prologue, gen, epilogue kind}
 * equal info5 (one kernel symbol; the others launch without events); NULL =
 * every launch. */
int vqx_probe_select(const int32_t* info5);
int vqx_probe_clear(void);
int vqx_probe_count(int64_t* n);
int vqx_probe_read(int64_t i, int32_t* info5, double* flops, float* ms);

/* A stream on all but `reserve_cus` of the current device's CUs
 * (hipExtStreamCreateWithCUMask; mask bit i is CU i / 8 of XCD i % 8, so
 * the top `reserve_cus` bits are cleared: reserve_cus / 8 per XCD), for measuring what co-resident work such as RCCL's all-reduce
 * kernels costs the step (bench.py --reserve-cus).  *cus_used = the CUs the
 * stream may use.  No reference counterpart (measurement only). */
int vqx_stream_create_cu_mask(int32_t reserve_cus, vqx_stream_t* out, int32_t* cus_used);
int vqx_stream_destroy(vqx_stream_t stream);

/* Host mailbox for the step statistics (ABI 127; replaces the loss .item()
 * reads of vqvae.py:85-87 / layers_vq.py:229-232 with one stream-ordered
 * publish the host polls).  vqx_mailbox_create allocates `slots` slots of
 * `floats` (<= 64) f32 values in mapped, coherent pinned host memory: layout
 * [slots] uint32 sequence numbers, then [slots][floats] values, zeroed; *host
 * is the host view, *dev the device pointer of the same bytes.
 * vqx_mailbox_publish (one 64-thread workgroup on `stream`) copies src[0..n)
 * into slot `slot` (and into dev_copy, a device buffer, when non-NULL), then,
 * behind a system-scope release, stores `seq` as the slot's sequence number:
 * a host that reads the number equal to seq reads that step's values.  No
 * marker or copy enters the stream. */
int vqx_mailbox_create(int32_t slots, int32_t floats, void** host, void** dev);
int vqx_mailbox_destroy(void* host);
int vqx_mailbox_publish(const float* src, int32_t n, float* dev_copy, void* box_dev, int32_t slot, int32_t slots,
                        int32_t floats, uint32_t seq, vqx_stream_t stream);

/* ABI version (major*100 + minor); VQX_ABI_VERSION is what this header describes. */
#define VQX_ABI_VERSION 128
int vqx_version(void);

#ifdef __cplusplus
}
#endif
#endif /* VQX_H */
