"""The VQ-VAE training step on MI355X: every arithmetic op of the reference's
hot path is a libvqx HIP kernel launched here on
torch's current stream; torch is used only for device memory and streams.

Step anatomy (frame-major activations [N = B*T, C], see include/vqx.h):

  pack     weight norm of every conv -> packed effective weights (1 launch pair)
  encoder  per resolution stage: stage conv (stride 1, or the strided
           down-sampler run as a 3-tap conv on s-frame-folded rows) | blocks
           {stack_layers x (conv (dilation 2**j on the first) -> GN stats
           [-> GN + LeakyReLU]) -> 1x1 skip conv with the last GroupNorm-apply
           + residual fused in its epilogue} | 1x1 out conv (f32 out).  Each
           GEMM producing c also stores LeakyReLU(c), so no GEMM applies an
           activation to its staged operands                      (vqvae.py:122-217)
  vq       distance/argmin/gather/commitment kernel + EMA statistics
                                                                 (layers_vq.py:268-323)
  decoder  per stage: ConvT (stride 1, or the strided up-sampler run as the
           adjoint of a folded 3-tap conv) | blocks {ConvT k (dilation 2**j;
           + speaker term as a per-utterance row bias) -> GN stats ->
           GN+tanh*sigmoid -> 1x1 res/skip conv with the residual add and the
           skip accumulation split in its epilogue} |
           ReLU(s*skip) -> 1x1 (ReLU epilogue) -> 1x1            (vqvae.py:220-343)
  loss     log-likelihood + its gradient in one pass            (layers.py:283-296)
  backward encoder (driven only by beta*commitment, the reference quirk:
           z_vq carries no gradient, layers_vq.py:315) and decoder: dgrad GEMMs
           with activation-derivative / residual epilogues, wgrad split-K slabs
           reduced by the weight-norm backward, GN backward (2 passes).
  update   global grad norm -> fused clip + Adam (+ StepLR on device); EMA codebook.

The recipe topologies (one stage, stack_layers 1, no dilation, kernel 3) run
exactly the fused schedule tuned for them; the general topology of vqvae.py
(several stages, resampling, dilation, stack_layers > 1, kernel 5) runs the
same kernels with the fusions that stay valid for each stage's shape.

The engine owns flat fp32 buffers for parameters, gradients and Adam moments;
model parameters are views into them, so `model.state_dict()` stays the
reference's and the optimizer touches one contiguous buffer.
"""
import bisect
import math
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import _lib as L
from .. import ops

F32 = torch.float32
KIND_CONV, KIND_CONVT, KIND_DOWN, KIND_UP = 0, 1, 3, 4


@dataclass(eq=False)
class ConvLayer:
    """One conv of the model as the stride-1 GEMM it runs as.
    kind 0 Conv1d / 1 ConvTranspose1d (flipped-tap conv, pad (k-1)*dil - p) /
    3 strided Conv1d (down-sampler) / 4 strided ConvTranspose1d (up-sampler):
    kinds 3-4 fold `scale` frames into channels (x'[u] = x[s*u .. s*u+s-1])
    and run a 3-tap, pad-1 conv (include/vqx.h VQX_WN_RESAMPLE)."""
    mod: object
    name: str
    kind: int
    cin: int
    cout: int
    k: int
    pad: int
    dil: int = 1
    scale: int = 1
    wp: torch.Tensor = None     # packed effective weight [rows, cols] (kinds 0/1: [cout, k*cin])
    norm: torch.Tensor = None   # ||v_o||
    slab: torch.Tensor = None   # wgrad partials [splits, rows, cols]
    splits: int = 1
    fix_dw: torch.Tensor = None   # wgrad_fixup: the in-launch reduced fp32 weight gradient [rows, cols]
    fix_cnt: torch.Tensor = None  # ... and its per-tile arrival counters
    btile: torch.Tensor = None  # kind 4: bias tiled over the s folded frames [s*cout]

    @property
    def rows(self):
        return self.cin if self.kind in (KIND_CONVT, KIND_UP) else self.cout

    @property
    def cols(self):
        if self.kind == KIND_DOWN:
            return 3 * self.scale * self.cin
        if self.kind == KIND_UP:
            return 3 * self.scale * self.cout
        return (self.cout if self.kind == KIND_CONVT else self.cin) * self.k


@dataclass
class EncBlock:
    """Conv1d_Layernorm_LRelu_Residual (layers.py:129-178)."""
    key: tuple
    convs: list
    gns: list
    skip: ConvLayer


@dataclass
class EncStage:
    conv: ConvLayer
    scale: int
    C: int
    blocks: list = field(default_factory=list)
    L: int = 1


@dataclass
class DecBlock:
    """DeConv1d_Layernorm_GLU_ResSkip (layers.py:181-249)."""
    key: tuple
    gidx: int            # position among all decoder blocks (skip accumulation order)
    conv_in: ConvLayer
    gn: object
    cond: ConvLayer
    rs: ConvLayer


@dataclass
class DecStage:
    conv: ConvLayer
    scale: int
    C: int
    blocks: list = field(default_factory=list)


def _tm(N):
    return (N + L.CONV_TILE_ROWS - 1) // L.CONV_TILE_ROWS


def _wn_block_bytes(e):
    """Approximate HBM bytes one workgroup of vqx_weight_norm_bwd moves for a
    table entry (csrc/vqx_misc.hip wn_bwd_kernel): a column-reduce block
    reads 32 columns of every partial row; a row block reads the row's
    split-K slabs and v and writes dv (four rows per block on the 1x1
    wave-per-row path)."""
    if e["kind"] == L.WN_COLREDUCE:
        return e["cin"] * 32 * 4
    rows_cout = e["kind"] in (0, L.WN_RESAMPLE)
    other = e["cin"] if rows_cout else e["cout"]
    cols = 3 * e.get("stride", 1) * other if e["kind"] in (L.WN_RESAMPLE, L.WN_RESAMPLE_T) else other * e["k"]
    sl = e.get("slabs")
    es = sl.element_size() if sl is not None else 4
    b = cols * (e.get("splits", 1) * es + 8)
    wave_rows = e["kind"] == 0 and e["k"] == 1 and e["cin"] <= 256 and (e["cin"] // 4) * e.get("splits", 1) <= 256
    return 4 * b if wave_rows else b


@dataclass
class EngineOptions:
    """Schedule choices of the engine.  The defaults are the measured-best
    configuration; A/B runs pass others through the model
    config's `engine` mapping (Model(arch), arch["engine"] = {...}), never
    through the environment.
      fuse_gn          GroupNorm statistics from GEMM epilogue tiles (False:
                       standalone statistics kernels)
      enc_gn_finalize  encoder GroupNorm statistics through a separate finalize
                       launch instead of the skip GEMM's in-launch merge
      side_stream      conditioning linears and EMA statistics + codebook update
                       on a second stream (measured 0.5-0.8% slower)
      wgrad_wgs, wgrad_wgs_1x1, wgrad_wgs_solo
                       workgroups per weight-gradient launch (the split-K
                       factor) of the 3-tap layers, the 1x1 layers and the
                       stage convs; wgrad_min_k: fewest frames per split
      wn_bwd_batch     the backward groups' weight-norm backward + bias
                       reductions batched (each group's split-K slabs and
                       partial sums kept in buffers of their own): one process
                       runs them all in one launch after the backward; data
                       parallel runs them every wn_bwd_ddp_groups groups, so
                       the all-reduce of each chunk's gradients still overlaps
                       the rest of the backward
      wn_bwd_ddp_groups  groups per batched launch under data parallelism
      lazy_stats       the step's loss statistics snapshotted on the device
                       and copied to the host when first read (trainer/
                       basic.py LazyLossDetail) instead of an eager D2H
      wn_bwd_sort      a batched launch's entries ordered by bytes per
                       workgroup, heaviest first (the last workgroups of the
                       flat grid are then short ones)
      slab_f32         fp32 split-K slabs in bf16 runs (+3.3% step time,
                       profiles/r04/slab_wfirst_ab.txt)
      fuse_grad_norm   one process, batched weight-norm backward: the global
                       gradient norm of the clip from sum-of-squares partials
                       the weight-norm backward leaves as it writes the
                       gradients (plus the few parameters it does not write),
                       instead of a pass re-reading the 125 MB gradient
      fuse_adam_wn     Adam writes the next forward's weight-norm row norms and
                       Conv1d packed weights as it updates weight_v / weight_g
                       (vqx_adam_step_wn); the forward then packs only the
                       ConvTranspose layers
      kernel_policy    include/vqx.h VQX_POLICY_* of every conv GEMM call (5:
                       the 1x1 layers on the two-workgroups-per-CU kernels
                       of round 4; automatic: three per CU)
      wgrad_fixup      the 3-tap layers' split-K weight-gradient slabs summed
                       inside the GEMM launch by the last split of each tile
                       (vqx_wgrad_args.fixup_dw, ABI 127): the weight-norm
                       backward then reads one fp32 gradient instead of the
                       bf16 slabs; bit-identical results
      early_stats      (lazy_stats) the loss statistics snapshotted at the end
                       of the forward, where they are final, so a host read
                       waits for the forward only (False: at the end of the
                       step, the read waits for the whole step)
      debug_checks     out-of-extent write detection (vae_npvc_amd/debug.py):
                       every engine buffer between guard canaries checked
                       after every libvqx call, and host extent checks of
                       every pointer argument; slow, for audits only
      fused_prologue   the training forward's three independent first jobs
                       (ConvT weight packs, conditioning linears, input
                       transpose) as one launch (vqx_step_prologue) when the
                       last optimizer step left the row norms current; the
                       same bits as the three launches
      bwd_streams      (one process) the encoder backward on a second stream
                       beside the decoder backward: the two chains share no
                       data (the decoder input carries no gradient), so their
                       launches fill each other's ramps and tails; the same
                       bits
      enc_bwd_early    (with bwd_streams, Trainer/engine train_step) the encoder
                       backward issued on the second stream right after the
                       VQ forward, beside the decoder forward and backward:
                       it needs only z, the gathered codes and the encoder's
                       activations; the same bits
      wn_bwd_split     (one process, batched) the encoder groups' weight-norm
                       backward as its own launch right after the encoder
                       backward (beside the decoder's under bwd_streams):
                       neutral, off (profiles/r06/bwd_streams_ab.txt)
      fused_close      the forward's closing work -- the log-loss and
                       commitment sums, the step statistics' mailbox publish --
                       in the EMA update's last workgroup
                       (vqx_vq_ema_update_close): two one-workgroup launches
                       fewer, the same bits"""
    fuse_gn: bool = True
    enc_gn_finalize: bool = False
    side_stream: bool = False
    wgrad_wgs: int = 256
    wgrad_wgs_1x1: int = 256
    wgrad_wgs_solo: int = 512
    wgrad_min_k: int = 512
    slab_f32: bool = False
    wn_bwd_batch: bool = True
    wn_bwd_ddp_groups: int = 5
    wn_bwd_sort: bool = True
    lazy_stats: bool = True
    fuse_grad_norm: bool = True
    fuse_adam_wn: bool = True
    kernel_policy: int = 0
    debug_checks: bool = False
    wgrad_fixup: bool = False
    early_stats: bool = True
    fused_prologue: bool = True
    fused_close: bool = True
    bwd_streams: bool = True
    wn_bwd_split: bool = False
    enc_bwd_early: bool = True
    side_priority: int = 0
    vq_stats_side: bool = False
    bwd_streams_ddp: bool = True


class _Stage:
    """Per-stage activation buffers of a Workspace."""


class Workspace:
    """All activations / gradients of one (B, T) shape (allocated once)."""

    def __init__(self, eng, B, T, train=True):
        d, cd, dev = eng.dims, eng.cd, eng.device
        self.B, self.T, self.N = B, T, B * T
        e = lambda *s, dt=cd: eng._empty(*s, dtype=dt)  # noqa: E731
        Z, S, Fo, mel, K = d["Z"], d["S"], d["F"], d["mel"], d["K"]
        fuse_opt = eng.opt.fuse_gn
        self.x = e(self.N, mel)
        # ---- encoder stages
        self.enc = []
        Tc = T
        for st in eng.enc_stages:
            if Tc % st.scale:
                raise ValueError(f"utterance length {Tc} is not a multiple of the down-sampling scale {st.scale}")
            Tc //= st.scale
            sw = _Stage()
            sw.T, sw.N, sw.C = Tc, B * Tc, st.C
            N, C, nb = sw.N, sw.C, len(st.blocks)
            sw.c = [e(N, C) for _ in range(nb + 1)]
            sw.a = [e(N, C) for _ in range(nb + 1)]   # LeakyReLU(c_j), written by the producing GEMM (ACT2)
            sw.h = [[e(N, C) for _ in range(st.L)] for _ in range(nb)]
            sw.g = [[e(N, C) for _ in range(st.L - 1)] for _ in range(nb)]  # LeakyReLU(GN(h)) of inner layers
            sw.mr = [[e(B, 2, dt=F32) for _ in range(st.L)] for _ in range(nb)]
            sw.fuse = Tc % 128 == 0 and C % 128 == 0 and fuse_opt
            if train:
                # colsum partials of dL/dc_j (the producing dgrad's COLSUM epilogue)
                sw.cs = [e(_tm(N), C, dt=F32) for _ in range(nb + 1)]
            self.enc.append(sw)
        self.Tz, self.Nz = Tc, B * Tc
        Nz = self.Nz
        self.z = e(Nz, Z, dt=F32)
        self.idx = torch.empty(Nz, device=dev, dtype=torch.int64)
        self.zq = e(Nz, Z, dt=F32)
        self.zq_c = e(Nz, Z)
        self.zq_j = e(Nz, Z) if d["jitter_p"] > 0 else None
        self.src_t = torch.empty(Tc, device=dev, dtype=torch.int32)
        self.jittered = False
        if eng.plain:  # straight-through quantizer: normalised frames / codebook and their norms
            self.z_norm = e(Nz, Z, dt=F32)
            self.z_len = e(Nz, dt=F32)
            self.embn = e(K, Z, dt=F32)
            self.e_len = e(K, dt=F32)
            self.pv_part = e(Nz // 4 + 8, dt=F32)
        self.vq_part = e(ops.vq_workspace(Nz, K, train or eng.plain, Z), dt=F32)  # VQ partials (+ statistics slabs)
        # EMA statistics bundle (all-reduced as one buffer in data parallel)
        self.ema = e(K * Z + K + K * Z, dt=F32)
        self.bsum = self.ema[: K * Z].view(K, Z)
        self.bcnt = self.ema[K * Z: K * Z + K]
        self.rand_rows = self.ema[K * Z + K:].view(K, Z)
        self.ema_part = eng._zeros(ops.ema_workspace(K, Z), dtype=F32)  # vqx_vq_ema_update workspace (+ counter)
        self.yemb = e(B, d["ydim"], dt=F32)
        # ---- decoder stages
        self.dec = []
        Td = Tc
        for st in eng.dec_stages:
            Td *= st.scale
            sw = _Stage()
            sw.T, sw.N, sw.C = Td, B * Td, st.C
            N, C, nb = sw.N, sw.C, len(st.blocks)
            sw.xs = [e(N, C) for _ in range(nb + 1)]
            sw.u = [e(N, 2 * C) for _ in range(nb)]
            sw.g = [e(N, C) for _ in range(nb)]
            sw.mr = [e(B, 4, dt=F32) for _ in range(nb)]
            sw.condbias = [e(B, 2 * C, dt=F32) for _ in range(nb)]
            sw.fuse = Td % 128 == 0 and C % 128 == 0 and fuse_opt
            if train:
                sw.dr = [e(N, C + S) for _ in range(2)] if nb else None   # [dL/dx | dL/dskip] ping-pong
                sw.dx = e(N, C) if not nb else None                        # stages without blocks
                sw.cs = [e(_tm(N), C, dt=F32) for _ in range(nb + 1)]     # colsum partials of dL/dx_j
                # dL/dx_nb of the last stage is zero and no kernel writes its partials: zeroed
                # here once, not every step (earlier stages' are overwritten by the next stage's dgrad)
                sw.cs[-1].zero_()
                sw.cs_all = [e(B, 2 * C, dt=F32) for _ in range(nb)]      # per-utterance colsums of du
            self.dec.append(sw)
        if Td != T:
            raise ValueError(f"decoder output length {Td} != input length {T} (resampling scales do not cancel)")
        if eng.n_dec_blocks:
            Ts = self.dec[eng.skip_stage].T
            if any(sw.T != Ts for sw, st in zip(self.dec, eng.dec_stages) if st.blocks):
                raise ValueError("the decoder sums the skip outputs of all blocks: they must share one frame rate")
        self.Nskip = B * T
        self.skip32 = e(self.Nskip, S, dt=F32)
        self.a_skip = e(self.Nskip, S)                 # ReLU(sqrt(1/len(layers)) * skip)
        self.f1 = e(self.Nskip, S)                     # ReLU(final conv 1 output)
        self.xhat = e(self.N, Fo, dt=F32)
        self.xhat_nct = e(B, Fo, T, dt=F32)
        # scalars: 0 x_loss, 1 sqerr, 4..7 EMA diagnostics
        self.stats = eng._zeros(8, dtype=F32)
        # GroupNorm partials written by GEMM epilogues (GNSTATS / GNBWD tiles:
        # [N/128][column tile][4]) when T and the group widths are multiples of 128
        Cmax = max([sw.C for sw in self.enc] + [2 * sw.C for sw in self.dec] + [1])
        Nmax = max([sw.N for sw in self.enc] + [sw.N for sw in self.dec] + [self.N])
        self.gst = e(max(1, Nmax // 128) * ((Cmax + 127) // 128) * 4, dt=F32)
        self.loss_part = e(1024, dt=F32)
        self.gn_part = e(B * 2 * 8 * 3, dt=F32)
        if not train:
            return
        NCe = max([sw.N * sw.C for sw in self.enc] + [1])
        if eng.fin2_pad is not None:  # zero columns up to the padded K of the output conv's DGRAD
            self.dxhat_pad = eng._zeros(self.N, eng.fin2_pad[0], dtype=cd)
            self.dxhat = self.dxhat_pad[:, :Fo]
        else:
            self.dxhat = self.dxhat_pad = e(self.N, Fo)
        self.df1 = e(self.Nskip, S)
        NCd = max([sw.N * sw.C for sw in self.dec] + [1])
        self.dg_flat = e(NCd)
        self.du_flat = e(2 * NCd)
        self.gnb_part = e(max(B * 64 * 2, max(1, Nmax // 128) * ((Cmax + 127) // 128) * 4), dt=F32)
        self.gnb_part_enc = e(self.gnb_part.numel(), dt=F32)  # the encoder backward's own (EngineOptions.bwd_streams)
        Lmax = max([st.L for st in eng.enc_stages] + [1])
        # per-utterance GN-backward sums per stack layer: conv bias, GN weight, GN bias
        self.colsum_b = [e(B * 2 * Cmax, dt=F32) for _ in range(Lmax)]
        self.dgam_b = [e(B * 2 * Cmax, dt=F32) for _ in range(Lmax)]
        self.dbet_b = [e(B * 2 * Cmax, dt=F32) for _ in range(Lmax)]
        # ... per block when the weight-norm backward is batched (EngineOptions.wn_bwd_batch):
        # the column reductions then read them after the whole backward
        self.blk_parts = {}
        if eng.opt.wn_bwd_batch:
            for si, st in enumerate(eng.enc_stages):
                for j in range(len(st.blocks)):
                    self.blk_parts[("enc", si, j)] = {k: [e(B * self.enc[si].C, dt=F32) for _ in range(st.L)]
                                                      for k in ("colsum_b", "dgam_b", "dbet_b")}
            for si, st in enumerate(eng.dec_stages):
                for j in range(len(st.blocks)):
                    self.blk_parts[("dec", si, j)] = {k: [e(B * 2 * self.dec[si].C, dt=F32)]
                                                      for k in ("dgam_b", "dbet_b")}
        self.dz = e(Nz, Z)
        self.dzq = e(Nz, Z) if eng.plain else None  # decoder gradient w.r.t. its (jittered) input
        self.dc_flat = [e(NCe) for _ in range(2)]   # encoder dL/dc ping-pong (viewed per stage)
        self.dh_flat = e(NCe)
        self.dy_flat = e(NCe)                       # inner-layer gradients (stack_layers > 1)
        self.tmp_flat = e(NCe)
        self.dyemb = e(B, d["ydim"], dt=F32)
        self.cs_part = e(64 * max(Cmax, S + Cmax, mel, 1024), dt=F32)
        self.cs_part_enc = e(self.cs_part.numel(), dt=F32)
        self.cs_skip = e(_tm(self.Nskip), S, dt=F32)  # dL/dskip
        self.cs_f1 = e(_tm(self.Nskip), S, dt=F32)    # dL/d(final conv 1 output)
        # bias-gradient row-part sums of the encoder output conv (from dL/dz) and of the
        # output conv (from dL/dxhat), reduced by their group's weight-norm backward launch
        self.cs_eo = eng._zeros(ops.COMMIT_PARTS, Z, dtype=F32)  # rows past colsum_parts stay 0
        self.cs_f2 = e(ops.colsum_parts(self.N, Fo, cd), Fo, dt=F32)
        self.lin_part = e(max(len(g) * ((O + 63) // 64) for O, g in eng.cond_groups.items()) * B * d["ydim"]
                          if eng.cond_groups else 1, dt=F32)  # split-K partials of d(embedding)
        eng._build_bwd_tables(self)

    # flat scratch viewed at a stage's shape
    @staticmethod
    def view(flat, N, C):
        return flat[: N * C].view(N, C)


class VQVAEEngine:
    def __init__(self, model, device, compute_dtype="fp32", options=None):
        self.m = model
        self.opt = options if options is not None else EngineOptions()
        self.device = torch.device(device)
        self.cd = torch.bfloat16 if compute_dtype in ("bf16", "bfloat16") else F32
        self.dt = ops.dt_code(self.cd)
        L.load()
        self._guards = None
        if self.opt.debug_checks:
            from .. import debug
            self._guards = debug.GuardSet(self.device)
            ops.set_debug_checks(True)
            debug.install(self._guards)
            import weakref
            weakref.finalize(self, debug.uninstall, self._guards)
        enc, dec = model.encoder, model.decoder
        self.dims = d = dict(mel=enc.in_ch, Z=enc.z_ch, S=dec.skip_ch, F=dec.final_ch, cond=dec.cond_ch,
                             K=model.quantizer.z_num, ydim=model.embeds._embedding.weight.shape[1],
                             jitter_p=model.jitter.probability)
        if d["Z"] not in (64, 128, 256) or model.quantizer.z_dim != d["Z"]:  # Model's constructor refuses these
            raise NotImplementedError("the fused VQ kernels are built for z_dim 64, 128 or 256")
        # straight-through VectorQuantizer (use_ema: false)
        self.plain = not model.use_ema
        self.vq_normalize = bool(getattr(model.quantizer, "normalize", False)) if self.plain else False
        self._flatten()
        if self._guards is not None:
            self._adopt_buffers()
        self._build_layers()
        self._ws = {}
        self.opt_ready = False
        self._enc_gn_separate = self.opt.enc_gn_finalize
        # optional side stream for the latency-bound work off the GEMM chain: the
        # speaker conditioning linears (needed only by the decoder) and the EMA
        # codebook statistics + update (needed only by the next step).  Measured
        # 0.5-0.8% slower end to end (profiles/r02/side_stream_ab.txt: the small
        # kernels squeeze into the GEMMs' single round of workgroups), so off by
        # default (EngineOptions.side_stream)
        self._side_on = self.device.type == "cuda" and self.opt.side_stream
        self._side = None
        self._wn_active = False   # inside backward(): the weight-norm backward may be batched
        self._wn_pending = []     # groups whose weight-norm backward is batched and not yet run
        self._wn_done = set()     # ... and those already run in this backward
        self._sq_plan_ready = None  # gradient-norm partials of this backward (fuse_grad_norm)
        # fused Adam + weight-norm preparation (fuse_adam_wn): its plan, and the
        # flat_p version the packed weights / norms it wrote belong to
        self._adam_wn, self._adam_wn_built, self._packed_version = None, False, None
        self._mailbox = None  # host mailbox of the step statistics (early_stats)

    # ------------------------------------------------------------ allocation
    def _empty(self, *shape, dtype=F32):
        """Every engine buffer comes from here (guarded under debug_checks)."""
        if self._guards is not None:
            return self._guards.empty(*shape, dtype=dtype, label=f"{dtype} {tuple(shape)}")
        return torch.empty(*shape, device=self.device, dtype=dtype)

    def _zeros(self, *shape, dtype=F32):
        t = self._empty(*shape, dtype=dtype)
        t.zero_()
        return t

    def _adopt_buffers(self):
        """debug_checks: the quantizer's EMA buffers (written by the EMA update)
        moved between guards too."""
        q = self.m.quantizer
        for name in ("emb_sum", "emb_elem", "embeddings"):
            t = getattr(q, name, None)
            if isinstance(t, torch.Tensor) and t.device == self.device and name in q._buffers:
                q._buffers[name] = self._guards.adopt(t, f"quantizer.{name}")

    # ------------------------------------------------------------ parameters
    def _flatten(self):
        params = list(self.m.parameters())
        self.params = params
        total = sum(p.numel() for p in params)
        self.flat_p = self._empty(total, dtype=F32)
        self.flat_g = self._zeros(total, dtype=F32)
        self.gviews = {}
        off = 0
        with torch.no_grad():
            for p in params:
                n = p.numel()
                self.flat_p[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.flat_p[off:off + n].view_as(p)
                self.gviews[p] = self.flat_g[off:off + n].view_as(p)
                off += n
        self.n_params = total
        self._p_off = [o for _, o in self._offsets_of(params)]
        self._p0_ptr = params[0].data_ptr()
        enc_ids = {id(p) for p in self.m.encoder.parameters()}
        self.enc_end = sum(p.numel() for p in params if id(p) in enc_ids)
        if not all(id(p) in enc_ids for p in params[: len(enc_ids)]):
            raise ValueError("the encoder's parameters must come first in model.parameters() "
                             "(the flat gradient buffer is all-reduced encoder-first)")

    def params_intact(self):
        return self.params[0].data_ptr() == self._p0_ptr and all(
            p.data_ptr() == self.flat_p.data_ptr() + 4 * o for p, o in self._offsets())

    def _offsets(self):
        return self._offsets_of(self.params)

    @staticmethod
    def _offsets_of(params):
        off = 0
        for p in params:
            yield p, off
            off += p.numel()

    def g(self, p):
        return self.gviews[p]

    def _params_written(self, tensors):
        """Indices (flat order) of the parameters whose gradient views overlap
        any of `tensors` (views into flat_g; None entries are skipped)."""
        base = self.flat_g.data_ptr()
        hit = set()
        for t in tensors:
            if t is None or t.numel() == 0:
                continue
            lo = (t.data_ptr() - base) // 4
            if lo < 0 or lo >= self.n_params:
                continue
            hi = lo + t.numel()
            i = bisect.bisect_right(self._p_off, lo) - 1
            while i < len(self.params) and self._p_off[i] < hi:
                hit.add(i)
                i += 1
        return sorted(hit)

    # ---- data parallel: issue each gradient range's all-reduce when it is final
    DDP_MIN_RUN = 64 << 10  # floats; smaller ready runs wait (they may still grow) until the flush

    def _grads_reset(self):
        self._g_ready = [False] * len(self.params)
        self._g_issued = [False] * len(self.params)

    def _grads_final(self, idxs, flush=False):
        """Mark parameters' gradients final and launch async mean all-reduces
        over every maximal contiguous run of final, not yet reduced gradients
        (runs below DDP_MIN_RUN floats wait unless `flush`)."""
        if self.comm is None:
            return
        for i in idxs:
            self._g_ready[i] = True
        n, i = len(self.params), 0
        while i < n:
            if not self._g_ready[i] or self._g_issued[i]:
                i += 1
                continue
            j = i
            while j < n and self._g_ready[j] and not self._g_issued[j]:
                j += 1
            lo, hi = self._p_off[i], self._p_off[j - 1] + self.params[j - 1].numel()
            if flush or hi - lo >= self.DDP_MIN_RUN:
                self.comm.grads_ready(self.flat_g, lo, hi)
                for k in range(i, j):
                    self._g_issued[k] = True
            i = j

    # ------------------------------------------------------------ layers
    def _mk(self, mod, name, dtype=None):
        from ..model.resample import ResampleConv1d
        dev = self.device
        if isinstance(mod, ResampleConv1d):
            Lr = ConvLayer(mod, name, KIND_UP if mod.transposed else KIND_DOWN, mod.cin, mod.cout, 3, 1, 1,
                           mod.scale)
            Lr.wp = self._empty(Lr.rows, Lr.cols, dtype=dtype or self.cd)
            if Lr.kind == KIND_UP:
                Lr.btile = self._empty(mod.scale * mod.cout, dtype=F32)
        else:
            kind = KIND_CONVT if mod.transposed else KIND_CONV
            dil = getattr(mod, "dilation", 1)
            pad = (mod.k - 1) * dil - mod.padding if kind == KIND_CONVT else mod.padding
            if 2 * pad != (mod.k - 1) * dil:
                raise NotImplementedError(f"{name}: asymmetric padding (the output length would change)")
            Lr = ConvLayer(mod, name, kind, mod.cin, mod.cout, mod.k, pad, dil)
            Lr.wp = self._empty(Lr.cout, Lr.k * Lr.cin, dtype=dtype or self.cd)
        Lr.norm = self._empty(Lr.rows, dtype=F32)
        return Lr

    def _build_layers(self):
        m, d = self.m, self.dims
        from ..model.layers import ResidualBlock
        enc_seq, dec_layers = m.encoder.encode, m.decoder.layers
        # ---- encoder stages
        self.enc_stages = []
        starts = list(m.encoder.stage_index)
        for si, i0 in enumerate(starts):
            conv = self._mk(enc_seq[i0], f"encoder.encode.{i0}")
            st = EncStage(conv, conv.scale, conv.cout)
            i = i0 + 1
            while i < len(enc_seq) and isinstance(enc_seq[i], ResidualBlock):
                blk = enc_seq[i]
                pre = f"encoder.encode.{i}"
                convs = [self._mk(c, f"{pre}.stack.{3 * l + 1}") for l, c in enumerate(blk.convs)]
                st.blocks.append(EncBlock(("enc", si, len(st.blocks)), convs, list(blk.norms),
                                          self._mk(blk.skip_layer, f"{pre}.skip_layer")))
                st.L = blk.layers
                i += 1
            self.enc_stages.append(st)
        self.enc_out = self._mk(enc_seq[len(enc_seq) - 1], f"encoder.encode.{len(enc_seq) - 1}")
        # ---- decoder stages
        self.dec_stages = []
        starts = list(m.decoder.stage_index) + [len(dec_layers)]
        gidx = 0
        for si in range(len(starts) - 1):
            i0 = starts[si]
            conv = self._mk(dec_layers[i0], f"decoder.layers.{i0}")
            st = DecStage(conv, conv.scale, conv.cout)
            for i in range(i0 + 1, starts[si + 1]):
                blk = dec_layers[i]
                pre = f"decoder.layers.{i}"
                st.blocks.append(DecBlock(("dec", si, len(st.blocks)), gidx, self._mk(blk.conv_in, f"{pre}.conv_in"),
                                          blk.norm_layer, self._mk(blk.conv_cond, f"{pre}.conv_cond", F32),
                                          self._mk(blk.res_skip_layers, f"{pre}.res_skip_layers")))
                gidx += 1
            self.dec_stages.append(st)
        self.n_dec_blocks = gidx
        self.n_dec_layers = len(dec_layers)      # vqvae.py:316 scales by sqrt(1/len(self.layers))
        with_blocks = [i for i, st in enumerate(self.dec_stages) if st.blocks]
        if not with_blocks:
            raise NotImplementedError("decoder without ResSkip blocks (no skip outputs to sum)")
        if with_blocks[-1] != len(self.dec_stages) - 1:
            raise NotImplementedError("decoder whose last stage has no ResSkip blocks (its output is unused)")
        self.skip_stage = with_blocks[0]
        self.fin1 = self._mk(m.decoder.final_layer[1], "decoder.final_layer.1")
        self.fin2 = self._mk(m.decoder.final_layer[3], "decoder.final_layer.3")
        # The output conv's DGRAD has K = final_channels (80 mel), off the
        # 64-deep K-tiles: the generic-tile kernel ran it 22 us.  Its packed
        # weight gets zero rows up to a multiple of 64 (the pack and Adam write
        # only the real rows) and dL/dxhat zero columns (Workspace.dxhat_pad),
        # so the DGRAD runs on the regular tiles; everything else sees the
        # real rows and columns.
        f2 = self.fin2
        Fp = -(-f2.cout // 64) * 64
        self.fin2_pad = None
        if Fp != f2.cout and f2.kind == KIND_CONV and f2.k == 1 and not m.decoder.final_layer[3].transposed:
            full = self._zeros(Fp, f2.cin, dtype=f2.wp.dtype)
            f2.wp = full[:f2.cout]
            self.fin2_pad = (Fp, full)
        self.dec_blocks = [b for st in self.dec_stages for b in st.blocks]
        self.dec_cond = [b.cond for b in self.dec_blocks]
        # speaker-conditioning linears grouped by output width (one batched launch per group)
        self.cond_groups = {}
        for b in self.dec_blocks:
            self.cond_groups.setdefault(b.cond.cout, []).append(b)
        self.convs = [st.conv for st in self.enc_stages]
        for st in self.enc_stages:
            for b in st.blocks:
                self.convs += b.convs + [b.skip]
        self.convs += [self.enc_out] + [st.conv for st in self.dec_stages]
        for b in self.dec_blocks:
            self.convs += [b.conv_in, b.cond, b.rs]
        self.convs += [self.fin1, self.fin2]
        # split-K factors for the wgrad GEMMs: one full round of ~480-512
        # workgroups (2 per CU) at config 2 (64 x 256 frames), at least 512
        # frames per split (round 3: the few-tile layers -- encoder output,
        # final convs, stage convs -- at 32 instead of 64 splits, -0.4% per
        # step; profiles/r03/wgs_ab.txt).  Measured sweep (tools/gemm_bench.py
        # --sweep-splits) on 128 x 128 tiles: dec_in best at 5, enc k3 at 10,
        # res/skip at 24, enc skip at 32 -- exactly floor(512 / tiles).  The
        # tile count comes from the library (3-tap layers use the tap-reuse
        # kernel's 128 x 192 tiles).  Frame counts follow each stage's rate.
        # Round 3 (profiles/r03/wgs_ab.txt): with the 3-tap WGRAD inside the fused
        # DGRAD+WGRAD launch (512 DGRAD workgroups of its own), 256 split-K
        # workgroups for the 3-tap layers (dec conv_in 4 splits, enc k3 8) beat
        # 512: 5.43 vs 5.53 ms per step; the stage convolutions, whose WGRAD
        # runs alone (no DGRAD beside it), stay at 512.  Round 5
        # (profiles/r05/wgs_ab.txt): with the 1x1 DGRAD + WGRAD launch three
        # workgroups per CU, 256 for the 1x1 layers (16 splits, half the slab
        # bytes) beat 512 by 1.4%: the 512 DGRAD + 256 WGRAD workgroups are one
        # round of three per CU; 192 +0.9%, 128 +5%, 384 +2%.
        o = self.opt  # workgroups per wgrad launch of the 3-tap / 1x1 layers / stage convs (WGRAD alone)
        wg_target, wg_1x1, wg_solo = o.wgrad_wgs, o.wgrad_wgs_1x1, o.wgrad_wgs_solo
        solo = {id(st.conv) for st in self.enc_stages} | {id(st.conv) for st in self.dec_stages}
        min_k = o.wgrad_min_k  # frames per split at least (256: +0.4%, 1024: +1.9%)
        B_ref, T_ref = 64, 256
        rate = {}
        Tc = T_ref
        for st in self.enc_stages:
            Tc //= max(1, st.scale)
            rate[id(st.conv)] = (Tc, Tc * st.scale)   # (output frames, input frames) per utterance
            for b in st.blocks:
                for Lr in b.convs + [b.skip]:
                    rate[id(Lr)] = (Tc, Tc)
        rate[id(self.enc_out)] = (Tc, Tc)
        for st in self.dec_stages:
            rate[id(st.conv)] = (Tc * st.scale, Tc)
            Tc *= st.scale
            for b in st.blocks:
                for Lr in (b.conv_in, b.cond, b.rs):
                    rate[id(Lr)] = (Tc, Tc)
        rate[id(self.fin1)] = rate[id(self.fin2)] = (T_ref, T_ref)
        for Lr in self.convs:
            if Lr in self.dec_cond:
                Lr.splits = 1
                continue
            To, Ti = rate[id(Lr)]
            To, Ti = max(1, To), max(1, Ti)
            if Lr.kind == KIND_DOWN:
                n, T_, r, c, k, pad, dil = B_ref * To, To, Lr.cout, Lr.scale * Lr.cin, 3, 1, 1
            elif Lr.kind == KIND_UP:
                n, T_, r, c, k, pad, dil = B_ref * Ti, Ti, Lr.cin, Lr.scale * Lr.cout, 3, 1, 1
            else:
                r, c = (Lr.cin, Lr.cout) if Lr.kind == KIND_CONVT else (Lr.cout, Lr.cin)
                n, T_, k, pad, dil = B_ref * To, To, Lr.k, Lr.pad, Lr.dil
            tiles = ops.wgrad_tiles(n, T_, r, c, k, pad, self.dt, dil=dil, policy=self.opt.kernel_policy)
            wgs = wg_solo if id(Lr) in solo else wg_1x1 if Lr.k == 1 else wg_target
            Lr.splits = max(1, min(wgs // tiles, n // min_k))
        # slab arena: every group's slabs in a region of their own when the
        # weight-norm backward is batched (EngineOptions.wn_bwd_batch), else one
        # group's slabs at a time (reused group by group, L2/MALL-resident).
        # bf16 runs keep the conv slabs in bf16 (each split's fp32 partial rounded
        # once, summed in fp32 by the weight-norm backward): half the bytes of the
        # split-K round trip.  The conditioning linears write dW directly (fp32).
        groups = self._bwd_groups()
        bf_slabs = self.dt == L.VQX_BF16 and not self.opt.slab_f32
        sdt = {id(Lr): (torch.bfloat16 if bf_slabs and Lr not in self.dec_cond else F32)
               for grp in groups for Lr in grp}

        def nbytes(Lr):
            n = Lr.splits * Lr.rows * Lr.cols * (4 if sdt[id(Lr)] == F32 else 2)
            return (n + 255) // 256 * 256

        # batched weight-norm backward (EngineOptions.wn_bwd_batch): every group's
        # slabs in a region of their own, all read by one launch after the backward
        per_group = [sum(nbytes(Lr) for Lr in grp) for grp in groups]
        arena = sum(per_group) if self.opt.wn_bwd_batch else max(per_group)
        self.arena = self._empty(arena, dtype=torch.uint8)
        base = 0
        for gi, grp in enumerate(groups):
            off = base
            if self.opt.wn_bwd_batch:
                base += per_group[gi]
            for Lr in grp:
                n = Lr.splits * Lr.rows * Lr.cols * (4 if sdt[id(Lr)] == F32 else 2)
                Lr.slab = self.arena[off:off + n].view(sdt[id(Lr)]).view(Lr.splits, Lr.rows, Lr.cols)
                off += nbytes(Lr)
        self.wn_fwd_table = ops.wn_table([self._wn_entry(Lr, bwd=False) for Lr in self.convs])
        self.groups = groups
        # in-launch split-K reduction of the 3-tap weight gradients (EngineOptions.wgrad_fixup):
        # an fp32 gradient buffer and tile counters per candidate layer; whether a call takes it
        # depends on the workspace's frames (Workspace.fix, _build_bwd_tables)
        if self.opt.wgrad_fixup and bf_slabs:
            for grp in groups:
                for Lr in grp:
                    if Lr.kind in (KIND_CONV, KIND_CONVT) and Lr.k == 3 and Lr.splits > 1:
                        Lr.fix_dw = self._empty(Lr.rows, Lr.cols, dtype=F32)
                        Lr.fix_cnt = self._zeros(((Lr.rows + 127) // 128) * (Lr.cols // 64 + 1), dtype=torch.int32)

    def _bwd_groups(self):
        gr = [[self.fin1, self.fin2]]
        for st in reversed(self.dec_stages):
            gr += [[b.conv_in, b.rs] for b in reversed(st.blocks)]
            gr += [[st.conv]]
        gr += [list(self.dec_cond), [self.enc_out]]
        for st in reversed(self.enc_stages):
            gr += [b.convs + [b.skip] for b in reversed(st.blocks)]
            gr += [[st.conv]]
        return gr

    def _wn_entry(self, Lr, bwd, fix=False):
        mod = Lr.mod
        if Lr.kind in (KIND_DOWN, KIND_UP):
            wn = mod.has_weight_norm
            e = dict(v=mod.v_param, g=mod.g_param, w_packed=Lr.wp, norm=Lr.norm,
                     kind=L.WN_RESAMPLE_T if Lr.kind == KIND_UP else L.WN_RESAMPLE, cout=mod.cout, cin=mod.cin,
                     k=mod.k, dtype=ops.dt_code(Lr.wp.dtype), splits=Lr.splits, stride=mod.scale, pad=mod.padding)
        else:
            wn = mod.has_weight_norm
            v = mod.weight_v if wn else mod.weight
            e = dict(v=v, g=mod.weight_g if wn else None, w_packed=Lr.wp, norm=Lr.norm, kind=Lr.kind, cout=Lr.cout,
                     cin=Lr.cin, k=Lr.k, dtype=ops.dt_code(Lr.wp.dtype), splits=Lr.splits)
        if bwd:
            v = e["v"]
            e.update(dv=self.g(v), dg=self.g(mod.weight_g) if wn else None, slabs=Lr.slab)
            if fix:  # the GEMM launch left the reduced fp32 gradient: one "slab"
                e.update(slabs=Lr.fix_dw.view(1, Lr.rows, Lr.cols), splits=1)
        return e

    def refresh_tables(self):
        """Rebuild descriptor tables (after remove_weight_norm or a re-flatten)."""
        self.wn_fwd_table = ops.wn_table([self._wn_entry(Lr, bwd=False) for Lr in self.convs])
        self._adam_wn, self._adam_wn_built, self._packed_version = None, False, None
        for (_, _, train), w in self._ws.items():
            if train:
                self._build_bwd_tables(w)

    def _bias_partials(self, w, producer_folded, buf):
        """COLSUM partial rows of a gradient tensor: the producing GEMM's row
        tiles, or one row of a standalone colsum when the producer is a folded
        (resampling) GEMM whose epilogue cannot sum unfolded columns."""
        return buf[:1] if producer_folded else buf

    def _fixup_layers(self, w):
        """{id(layer)} of the 3-tap layers whose weight gradient takes the
        in-launch split-K reduction at this workspace's frames."""
        on = set()
        pol, sdt = self.opt.kernel_policy, L.VQX_BF16
        for si, st in enumerate(self.enc_stages):
            sw = w.enc[si]
            for b in st.blocks:
                for Lr in b.convs:
                    if Lr.fix_dw is not None and Lr.kind == KIND_CONV and ops.wgrad_fixup_ok(
                            sw.N, sw.T, Lr.cout, Lr.cin, Lr.k, Lr.pad, self.dt, sdt, dil=Lr.dil, policy=pol):
                        on.add(id(Lr))
        for si, st in enumerate(self.dec_stages):
            sw = w.dec[si]
            for b in st.blocks:
                Lr = b.conv_in
                if Lr.fix_dw is not None and Lr.kind == KIND_CONVT and ops.wgrad_fixup_ok(
                        sw.N, sw.T, Lr.cin, Lr.cout, Lr.k, Lr.pad, self.dt, sdt, dil=Lr.dil, policy=pol):
                    on.add(id(Lr))
        return on

    def _build_bwd_tables(self, w):
        """Per-workspace backward tables: each group's weight-norm backward plus
        the column reductions of the bias / GroupNorm-affine partials that are
        final when the group's GEMMs are done (one launch per group)."""
        B, S = w.B, self.dims["S"]
        g = self.g
        cr = ops.colreduce_entry
        w.fix = self._fixup_layers(w) if self.opt.wgrad_fixup else set()

        def wb(Lr):  # a layer's backward entry (its reduced fp32 gradient when w.fix has it)
            return self._wn_entry(Lr, True, fix=id(Lr) in w.fix)

        t = {}
        t["fin"] = [wb(self.fin1), wb(self.fin2),
                    cr(w.cs_f1, g(self.fin1.mod.bias)), cr(w.cs_f2, g(self.fin2.mod.bias))]
        ns = len(self.dec_stages)
        for si, st in enumerate(self.dec_stages):
            sw = w.dec[si]
            C2 = 2 * sw.C
            nb = len(st.blocks)
            for j, b in enumerate(st.blocks):
                dg_b = self._bview(self._blk(w, "dec", si, j, "dgam_b", 0), B, C2)
                db_b = self._bview(self._blk(w, "dec", si, j, "dbet_b", 0), B, C2)
                rb = g(b.rs.mod.bias)
                # dL/dx_{j+1}: zero after the last block of the last stage (cs zeroed), else the
                # colsums of the next block's / next stage conv's dgrad
                nxt_folded = (j == nb - 1 and si + 1 < ns and self.dec_stages[si + 1].conv.kind == KIND_UP)
                t[b.key] = [wb(b.conv_in), wb(b.rs),
                            cr(self._bias_partials(w, nxt_folded, sw.cs[j + 1]), rb[:sw.C]), cr(w.cs_skip, rb[sw.C:]),
                            cr(sw.cs_all[j], g(b.conv_in.mod.bias)), cr(dg_b, g(b.gn.weight)), cr(db_b, g(b.gn.bias))]
            first_folded = not st.blocks and si + 1 < ns and self.dec_stages[si + 1].conv.kind == KIND_UP
            t[("dec_stage", si)] = [wb(st.conv),
                                    cr(self._bias_partials(w, first_folded, sw.cs[0]), g(st.conv.mod.bias))]
        t["cond"] = [wb(Lr) for Lr in self.dec_cond]
        t["enc_out"] = [wb(self.enc_out), cr(w.cs_eo, g(self.enc_out.mod.bias))]
        ne = len(self.enc_stages)
        for si, st in enumerate(self.enc_stages):
            sw = w.enc[si]
            C = sw.C
            nb = len(st.blocks)
            for j, b in enumerate(st.blocks):
                # dL/dc_{j+1} comes from the next block's skip dgrad, the next stage conv's
                # dgrad (folded when it down-samples) or the output conv's dgrad
                nxt_folded = j == nb - 1 and si + 1 < ne and self.enc_stages[si + 1].conv.kind == KIND_DOWN
                ent = [wb(Lr) for Lr in b.convs] + [wb(b.skip), cr(self._bias_partials(w, nxt_folded, sw.cs[j + 1]),
                                                                    g(b.skip.mod.bias))]
                for l, (Lr, gn) in enumerate(zip(b.convs, b.gns)):
                    ent += [cr(self._bview(self._blk(w, "enc", si, j, "colsum_b", l), B, C), g(Lr.mod.bias)),
                            cr(self._bview(self._blk(w, "enc", si, j, "dgam_b", l), B, C), g(gn.weight)),
                            cr(self._bview(self._blk(w, "enc", si, j, "dbet_b", l), B, C), g(gn.bias))]
                t[b.key] = ent
            first_folded = not st.blocks and si + 1 < ne and self.enc_stages[si + 1].conv.kind == KIND_DOWN
            t[("enc_stage", si)] = [wb(st.conv),
                                    cr(self._bias_partials(w, first_folded, sw.cs[0]), g(st.conv.mod.bias))]
        w.bwd_tables = {k: ops.wn_table(v) for k, v in t.items()}
        w.bwd_entries = t
        w.bwd_table_cache = {}  # group sequence -> table of one batched launch (_wn_run)
        w.bwd_ents_cache = {}   # ... its entries and gradient-norm partial count
        w.bwd_sq_cache = {}     # the launches of a backward -> their gradient-norm plan (_sq_finish)
        w.sq_buf = None
        # parameters whose gradients are final once a group's launch is done
        # (data parallel: their all-reduce is issued right then, parallel/ddp.py)
        w.bwd_params = {k: self._params_written([t_ for e in entries for t_ in (e.get("dv"), e.get("dg"))])
                        for k, entries in t.items()}
        # all ResSkip blocks' conditioning linears, forward and backward, one table per output width
        w.cond_tables = {}
        for O, blocks in self.cond_groups.items():
            ents = []
            for b in blocks:
                si, j = b.key[1], b.key[2]
                sw = w.dec[si]
                ents.append(dict(W=b.cond.wp, bias=b.cond.mod.bias, out=sw.condbias[j], dout=sw.cs_all[j],
                                 dW=b.cond.slab.view(b.cond.rows, b.cond.cols), dbias=g(b.cond.mod.bias)))
            w.cond_tables[O] = ops.linear_table(ents)

    MAX_EVAL_WS = 4  # inference over variable-length utterances keeps only the latest shapes

    def ws(self, B, T, train=True):
        key = (B, T, train)
        w = self._ws.get(key)
        if w is None:
            if train and (B, T, False) in self._ws:
                del self._ws[(B, T, False)]
            if not train:
                evals = [k for k in self._ws if not k[2]]
                for k in evals[: max(0, len(evals) - self.MAX_EVAL_WS + 1)]:
                    del self._ws[k]
            w = self._ws[key] = Workspace(self, B, T, train)
        elif not train:
            self._ws[key] = self._ws.pop(key)  # most recently used last
        return w

    # ------------------------------------------------------------ conv helpers
    def fwd(self, Lr, x, y, T, **kw):
        """y = conv(x); T = frames per utterance of the input x."""
        kw["policy"] = self.opt.kernel_policy
        if Lr.kind in (KIND_CONV, KIND_CONVT):
            ops.conv_fwd(x, Lr.wp, y, T=T, cin=Lr.cin, cout=Lr.cout, ntaps=Lr.k, pad=Lr.pad, dil=Lr.dil, **kw)
        elif Lr.kind == KIND_DOWN:
            s = Lr.scale
            ops.conv_fwd(x.view(-1, s * Lr.cin), Lr.wp, y, T=T // s, cin=s * Lr.cin, cout=Lr.cout, ntaps=3, pad=1,
                         **kw)
        else:  # up-sampler: the adjoint of the folded conv, bias tiled over the s output frames
            s = Lr.scale
            if kw.get("bias") is not None:
                kw["bias"] = Lr.btile
            ops.conv_dgrad(x, Lr.wp, y.view(-1, s * Lr.cout), T=T, cin=Lr.cin, cout=s * Lr.cout, ntaps=3, pad=1,
                           **kw)

    def dgrad(self, Lr, dy, dx, T, **kw):
        """dx = dL/d(input) from dy = dL/d(output); T = frames per utterance of dy."""
        kw["policy"] = self.opt.kernel_policy
        if Lr.kind in (KIND_CONV, KIND_CONVT):
            ops.conv_dgrad(dy, Lr.wp, dx, T=T, cin=Lr.cout, cout=Lr.cin, ntaps=Lr.k,
                           pad=(Lr.k - 1) * Lr.dil - Lr.pad, dil=Lr.dil, **kw)
        elif Lr.kind == KIND_DOWN:
            s = Lr.scale
            if kw.get("mask") is not None:
                kw["mask"] = kw["mask"].view(-1, s * Lr.cin)
            ops.conv_dgrad(dy, Lr.wp, dx.view(-1, s * Lr.cin), T=T, cin=Lr.cout, cout=s * Lr.cin, ntaps=3, pad=1,
                           **kw)
        else:
            s = Lr.scale
            ops.conv_fwd(dy.view(-1, s * Lr.cout), Lr.wp, dx, T=T // s, cin=s * Lr.cout, cout=Lr.cin, ntaps=3,
                         pad=1, **kw)

    _fix_now = frozenset()  # the current backward's workspace's Workspace.fix
    _side_pending = False  # work issued on the side stream since the last join

    def wgrad(self, Lr, dy, x, T, pro=L.PRO_NONE, scale=1.0):
        """Weight-gradient slabs from dy (output gradient, T frames per utterance) and the input x."""
        if id(Lr) in self._fix_now:
            raise RuntimeError(f"{Lr.name}: the in-launch split-K reduction runs through wgrad_dgrad only")
        pol = self.opt.kernel_policy
        if Lr.kind == KIND_CONV:
            ops.conv_wgrad(dy, x, Lr.slab, T=T, r_dim=Lr.cout, c_dim=Lr.cin, ntaps=Lr.k, pad=Lr.pad, dil=Lr.dil,
                           shift_sign=1, q_prologue=pro, pro_scale=scale, splits=Lr.splits, policy=pol)
            return
        if pro != L.PRO_NONE:
            raise ValueError(f"weight-gradient prologue {pro} is defined for plain convs only (layer kind {Lr.kind})")
        if Lr.kind == KIND_CONVT:
            ops.conv_wgrad(x, dy, Lr.slab, T=T, r_dim=Lr.cin, c_dim=Lr.cout, ntaps=Lr.k, pad=Lr.pad, dil=Lr.dil,
                           shift_sign=-1, splits=Lr.splits, policy=pol)
        elif Lr.kind == KIND_DOWN:
            s = Lr.scale
            ops.conv_wgrad(dy, x.view(-1, s * Lr.cin), Lr.slab, T=T, r_dim=Lr.cout, c_dim=s * Lr.cin, ntaps=3, pad=1,
                           shift_sign=1, splits=Lr.splits, policy=pol)
        else:
            s = Lr.scale
            ops.conv_wgrad(x, dy.view(-1, s * Lr.cout), Lr.slab, T=T // s, r_dim=Lr.cin, c_dim=s * Lr.cout, ntaps=3,
                           pad=1, shift_sign=1, splits=Lr.splits, policy=pol)

    def wgrad_dgrad(self, Lr, dy, x, dx, T, **kw):
        """self.wgrad(Lr, dy, x, T) then self.dgrad(Lr, dy, dx, T, **kw): for a plain
        Conv1d as one vqx_conv1d_dgrad_wgrad call (one launch interleaving both
        GEMMs where a fused kernel covers the layer)."""
        if Lr.kind not in (KIND_CONV, KIND_CONVT):
            self.wgrad(Lr, dy, x, T)
            self.dgrad(Lr, dy, dx, T, **kw)
            return
        pol = self.opt.kernel_policy
        dkw = dict(T=T, cin=Lr.cout, cout=Lr.cin, ntaps=Lr.k, pad=(Lr.k - 1) * Lr.dil - Lr.pad, dil=Lr.dil, policy=pol,
                   **kw)
        wkw = dict(T=T, ntaps=Lr.k, pad=Lr.pad, dil=Lr.dil, splits=Lr.splits, policy=pol)
        if id(Lr) in self._fix_now:  # the in-launch split-K reduction (EngineOptions.wgrad_fixup)
            wkw.update(fixup_dw=Lr.fix_dw, fixup_counters=Lr.fix_cnt)
        if Lr.kind == KIND_CONV:  # as self.wgrad
            ops.conv_dgrad_wgrad(dy, Lr.wp, dx, dkw, dy, x, Lr.slab, dict(wkw, r_dim=Lr.cout, c_dim=Lr.cin, shift_sign=1))
        else:
            ops.conv_dgrad_wgrad(dy, Lr.wp, dx, dkw, x, dy, Lr.slab, dict(wkw, r_dim=Lr.cin, c_dim=Lr.cout, shift_sign=-1))

    def bias_grad(self, part, dy, zero_tail=False):
        """First level of a conv bias gradient (the column sums of dy) into the
        first colsum_parts rows of `part` (the rest must be zero: `zero_tail`
        clears them); its group's weight-norm backward launch adds the rows (a
        VQX_WN_COLREDUCE entry, _build_bwd_tables)."""
        n = ops.colsum_parts(dy.shape[0], dy.shape[1], dy.dtype)
        ops.colsum_partials(dy, part[:n])
        if zero_tail and n < part.shape[0]:
            ops.zero_(part[n:])

    # ------------------------------------------------------------ forward
    def pack_weights(self):
        plan = self._adam_wn
        if plan is not None and self._packed_version == self._param_version():
            # the last optimizer step packed the Conv1d layers and wrote every
            # ConvT row norm for the current parameters (vqx_adam_step_wn)
            if plan[2] is not None:
                ops.weight_norm_fwd(plan[2], flags=plan[3])
            if self._guards is not None:  # debug_checks: the packed weights must be those of the parameters
                self._check_packed()
        else:
            ops.weight_norm_fwd(self.wn_fwd_table)
        self._up_bias()

    def _up_bias(self):
        for st in self.dec_stages:
            if st.conv.kind == KIND_UP:  # the up-sampler's bias, once per folded frame
                s = st.conv.scale
                ops.convert_2d(st.conv.mod.bias.detach().view(1, -1).expand(s, -1), st.conv.btile.view(s, -1))

    def _side_stream(self):
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device, priority=self.opt.side_priority)
        return self._side

    def _join(self):
        """Order the current stream after all side-stream work issued so far
        (the previous step's codebook update, its loss diagnostics); nothing to
        do when no work went there since the last join."""
        if self._side is not None and self._side_pending:
            torch.cuda.current_stream().wait_stream(self._side)
            self._side_pending = False

    def _fork(self):
        """The side stream, ordered after everything issued so far on the current stream."""
        side = self._side_stream()
        side.wait_stream(torch.cuda.current_stream())
        self._side_pending = True
        return side

    def _cond_ids(self, w, ids):
        """The conditioning linears read their input rows straight from the
        embedding table (linear_batched_*_ids: no lookup launch) for this batch."""
        emb = self.m.embeds._embedding.weight
        return (getattr(w, "cond_tables", None) is not None and bool(self.cond_groups) and ids.dtype == torch.int64
                and all(ops.linear_ids_ok(w.B, blocks[0].cond.cin, O, emb) for O, blocks in self.cond_groups.items()))

    def embed_and_cond(self, w, y):
        ids = y.reshape(-1)
        emb = self.m.embeds._embedding.weight
        w.cond_ids_mode = self._cond_ids(w, ids)
        if w.cond_ids_mode:
            for O, blocks in self.cond_groups.items():
                ops.linear_batched_fwd_ids(w.cond_tables[O], emb, ids, w.B, blocks[0].cond.cin, O)
            return
        ops.embedding_fwd(emb, ids, w.yemb)
        tabs = getattr(w, "cond_tables", None)
        for O, blocks in self.cond_groups.items():
            if tabs is not None:
                ops.linear_batched_fwd(tabs[O], w.yemb, w.B, blocks[0].cond.cin, O)
            else:
                for b in blocks:
                    ops.linear_f32(w.yemb, b.cond.wp, b.cond.mod.bias, w.dec[b.key[1]].condbias[b.key[2]])

    def _fused_prologue(self, w, x):
        """pack_weights + embed_and_cond + the encoder's input transpose as one
        launch (ops.step_prologue) when the shapes allow; False: nothing done."""
        plan = self._adam_wn
        if (not self.opt.fused_prologue or self._side_on or plan is None
                or self._packed_version != self._param_version() or not x.is_contiguous()):
            return False
        if plan[2] is not None and (len(plan[2][0]) > 256 or not (plan[3] & ops.WNF_NORMS_READY
                                                                  or all(e.kind != 1 for e in plan[2][0]))):
            return False  # the launch skips the ConvT norm pre-pass
        cond = None
        if len(self.cond_groups) == 1 and self._cond_ids(w, w.y_dev):
            (O, blocks), = self.cond_groups.items()
            w.cond_ids_mode = True
            cond = (w.cond_tables[O], self.m.embeds._embedding.weight, w.y_dev, w.B, blocks[0].cond.cin, O)
        else:  # several widths or a conditioning input the launch does not take: its own launches
            self.embed_and_cond(w, w.y_dev)
        ops.step_prologue(plan[2], cond, x, w.x)
        self._up_bias()
        if self._guards is not None:
            self._check_packed()
        self.n_fused_prologue = getattr(self, "n_fused_prologue", 0) + 1
        return True

    def encoder_fwd(self, w, x_nct, transposed=False):
        if not transposed:
            ops.nct_to_ntc(x_nct, w.x)
        inp, T_in = w.x, w.T
        for si, st in enumerate(self.enc_stages):
            sw = w.enc[si]
            T = sw.T
            # every GEMM producing c_j also writes a_j = LeakyReLU(c_j), the operand
            # of the next conv stack / stage conv / output conv (vqvae.py:171, layers.py:152)
            self.fwd(st.conv, inp, sw.c[0], T_in, bias=st.conv.mod.bias, act=L.PRO_LRELU, y2=sw.a[0])
            for j, b in enumerate(st.blocks):
                src = sw.a[j]
                gkw = {}
                for l, (Lr, gn) in enumerate(zip(b.convs, b.gns)):
                    h, mr = sw.h[j][l], sw.mr[j][l]
                    last = l == st.L - 1
                    if sw.fuse:  # statistics of h from the GEMM's epilogue tiles
                        self.fwd(Lr, src, h, T, bias=Lr.mod.bias, gn_stats=w.gst, gn_groups=1)
                        if last and not self._enc_gn_separate:
                            gkw = dict(gn_tiles=w.gst)  # merged inside the skip GEMM
                        else:
                            ops.gn_finalize_tiles(w.gst, sw.N, T, sw.C, 1, mr)
                    else:
                        self.fwd(Lr, src, h, T, bias=Lr.mod.bias)
                        ops.groupnorm_stats(h, T, 1, w.gn_part, mr)
                    if not last:  # LeakyReLU(GN(h)): the next conv's operand (layers.py:156-161)
                        ops.gn_lrelu_fwd(h, sw.g[j][l], T, mr, gn.weight, gn.bias)
                        src = sw.g[j][l]
                gn = b.gns[-1]
                self.fwd(b.skip, sw.c[j], sw.c[j + 1], T, bias=b.skip.mod.bias, gn_h=sw.h[j][-1], gn_mr=sw.mr[j][-1],
                         gn_gamma=gn.weight, gn_beta=gn.bias, act=L.PRO_LRELU, y2=sw.a[j + 1], **gkw)
            inp, T_in = sw.a[-1], T
        self.fwd(self.enc_out, inp, w.z, T_in, bias=self.enc_out.mod.bias, out_f32=True)

    def decoder_fwd(self, w, zq_c):
        inp, T_in = zq_c, w.Tz
        for si, st in enumerate(self.dec_stages):
            sw = w.dec[si]
            T, C = sw.T, sw.C
            self.fwd(st.conv, inp, sw.xs[0], T_in, bias=st.conv.mod.bias)
            for j, b in enumerate(st.blocks):
                ci, gn, rs = b.conv_in, b.gn, b.rs
                if sw.fuse:  # statistics from the GEMM's epilogue tiles, finalised inside the GLU launch
                    self.fwd(ci, sw.xs[j], sw.u[j], T, bias=ci.mod.bias, rowbias=sw.condbias[j], gn_stats=w.gst,
                             gn_groups=2)
                    ops.gn_glu_fwd_tiles(sw.u[j], sw.g[j], T, w.gst, sw.mr[j], gn.weight, gn.bias)
                else:
                    self.fwd(ci, sw.xs[j], sw.u[j], T, bias=ci.mod.bias, rowbias=sw.condbias[j])
                    ops.groupnorm_stats(sw.u[j], T, 2, w.gn_part, sw.mr[j])
                    ops.gn_glu_fwd(sw.u[j], sw.g[j], T, sw.mr[j], gn.weight, gn.bias)
                self.fwd(rs, sw.g[j], sw.xs[j + 1], T, bias=rs.mod.bias, res=sw.xs[j], out2=w.skip32, split_col=C,
                         out2_accumulate=(b.gidx > 0))
            inp, T_in = sw.xs[-1], T
        # final_layer = ReLU, conv, ReLU, conv on sqrt(1/len(layers)) * sum(skips) (vqvae.py:316-318)
        ops.scale_act_2d(w.skip32, w.a_skip, math.sqrt(1.0 / self.n_dec_layers), L.PRO_RELU)
        self.fwd(self.fin1, w.a_skip, w.f1, w.T, bias=self.fin1.mod.bias, act=L.PRO_RELU)
        self.fwd(self.fin2, w.f1, w.xhat, w.T, bias=self.fin2.mod.bias, out_f32=True)

    # ------------------------------------------------------------ quantizer host logic
    def _perm_rows(self, n, K, rank_offset=0, n_local=None):
        """torch.randperm(n)[:K] on the CPU generator (layers_vq.py:197,213),
        mapped to local row ids (-1 = row owned by another rank): a host int32
        tensor for ops.gather_rows_host, which passes it to the kernel by
        value (a host-to-device copy on the stream idled it ~5.5 us)."""
        perm = torch.randperm(n)[:K]
        if n_local is not None:
            from ..parallel.ddp import owned_rows
            perm = owned_rows(perm, rank_offset, n_local)
        return perm.to(torch.int32)

    def _tile_rows(self, w):
        """N < K path of _tile (layers_vq.py:183-190): repeat z with N(0, 0.01/sqrt(D))
        noise drawn on the CPU generator, then take perm rows.  Host side; rare.
        Data parallel: the tiling runs on the gathered GLOBAL batch (rank
        order = the single-process batch order), and every rank draws the same
        noise and permutation from its identically seeded CPU generator, so all
        ranks hold the single-process global-batch rows."""
        z = w.z.detach()
        if self.comm is not None:
            z = self.comm.all_gather_cat(z)
        z = z.cpu()
        n, dd = z.shape
        K = self.dims["K"]
        rep = (K + n - 1) // n
        zt = z.repeat(rep, 1)
        zt = zt + torch.randn_like(zt) * (0.01 / np.sqrt(dd))
        rows = zt[torch.randperm(zt.shape[0])][:K]
        return rows.to(self.device, non_blocking=False)

    def jitter_map(self, T):
        """Jitter (layers_vq.py:353-379): numpy-RNG neighbour map, consuming the
        global numpy stream exactly like np.random.choice (one uniform per
        choice).  Replaces with probability 1-p (the reference's indexing)."""
        p = self.dims["jitter_p"]
        src = np.arange(T, dtype=np.int32)
        cdf0 = np.cumsum([p, 1 - p])
        cdf0 = cdf0 / cdf0[-1]
        rs = np.random.random_sample
        for i in range(T):
            u = rs()
            choice = 1 if u < cdf0[0] else 0  # np.random.choice([1, 0], p=[p, 1-p])
            if choice == 0:  # [True, False][0] -> replace
                if i == 0:
                    src[i] = 1
                elif i == T - 1:
                    src[i] = T - 2
                else:
                    u2 = rs()
                    src[i] = i + (-1 if u2 < 0.5 else 1)
        return src

    # ------------------------------------------------------------ backward
    def _wn_batched(self):
        return self.opt.wn_bwd_batch and self._wn_active

    def _wn_bwd(self, w, key):
        """A backward group's weight-norm backward + bias/affine reductions;
        its gradients are final afterwards (data parallel: reduce them now).
        Batched: noted here and run with other groups' in one launch -- by
        _wn_bwd_flush after the backward (one process), or every
        wn_bwd_ddp_groups groups (data parallel, whose all-reduces start then)."""
        if self._wn_batched():
            self._wn_pending.append(key)
            if self.comm is not None and len(self._wn_pending) >= max(1, self.opt.wn_bwd_ddp_groups):
                self._wn_run(w)
            return
        ops.weight_norm_bwd(w.bwd_tables[key])
        self._grads_final(w.bwd_params[key])

    def _wn_run(self, w):
        """One launch for the pending groups (their tables concatenated, cached
        per group sequence), then their gradients are final.  One process
        (fuse_grad_norm): each launch also leaves its gradient-norm partials in
        the next part of the workspace's buffer (w.sq_buf; _sq_finish combines
        the launches of a backward)."""
        keys = tuple(self._wn_pending)
        self._wn_pending = []
        if not keys:
            return
        tab = w.bwd_table_cache.get(keys)
        if tab is None:
            ents = [e for k in keys for e in w.bwd_entries[k]]
            if self.opt.wn_bwd_sort:  # entries are independent: any order gives the same bits
                ents.sort(key=_wn_block_bytes, reverse=True)
            tab = w.bwd_table_cache[keys] = ops.wn_table(ents)
            w.bwd_ents_cache[keys] = (ents, ops.weight_norm_bwd_partials(tab))
        if self.comm is None and self.opt.fuse_grad_norm:
            n = w.bwd_ents_cache[keys][1]
            buf = self._sq_buf(w)
            off = self._sq_off
            if off + n > buf.numel():
                raise RuntimeError(f"gradient-norm partials: {off + n} > {buf.numel()}")
            ops.weight_norm_bwd(tab, sq_partials=buf[off:off + n])
            self._sq_off = off + n
            self._sq_runs.append(keys)
        else:
            ops.weight_norm_bwd(tab)
        self._wn_done.update(keys)
        self._grads_final([i for k in keys for i in w.bwd_params[k]])

    def _sq_buf(self, w):
        """Gradient-norm partials of every weight-norm backward entry (their
        counts add up entry by entry, so any split of the groups fits)."""
        if getattr(w, "sq_buf", None) is None:
            ents = [e for k in w.bwd_entries for e in w.bwd_entries[k]]
            w.sq_buf = self._zeros(max(1, ops.weight_norm_bwd_partials(ops.wn_table(ents))), dtype=F32)
        return w.sq_buf

    def _sq_finish(self, w):
        """The gradient-norm plan of this backward's weight-norm launches: their
        partials (w.sq_buf[:offset]) and the flat ranges none of them wrote."""
        runs = tuple(self._sq_runs)
        if not runs:
            return
        plan = w.bwd_sq_cache.get(runs, False)
        if plan is False:
            ents = [e for k in runs for e in w.bwd_ents_cache[k][0]]
            plan = w.bwd_sq_cache[runs] = self._sq_plan(ents, w.sq_buf[:self._sq_off])
        self._sq_plan_ready = plan

    def _sq_plan(self, ents, parts):
        """Gradient-norm plan of batched weight-norm backward launches:
        (their partials, int64 [n, 2] device ranges of the flat gradient the
        launches do not write).  None when their writes overlap (an element
        would be counted twice) -- the step then re-reads the gradient instead."""
        base = self.flat_g.data_ptr()
        iv = []
        for e in ents:
            for k in ("dv", "dg"):
                t = e.get(k)
                if t is None or t.numel() == 0:
                    continue
                lo = (t.data_ptr() - base) // 4
                if not t.is_contiguous() or lo < 0 or lo + t.numel() > self.n_params:
                    return None
                iv.append((lo, lo + t.numel()))
        iv.sort()
        rest, cur = [], 0
        for lo, hi in iv:
            if lo < cur:
                return None
            if lo > cur:
                rest.append((cur, lo - cur))
            cur = hi
        if cur < self.n_params:
            rest.append((cur, self.n_params - cur))
        rng = torch.tensor(rest, dtype=torch.int64).view(-1, 2).to(self.device) if rest else None
        return parts, rng

    def _wn_bwd_flush(self, w):
        if not self._wn_batched():
            return
        done = set(self._wn_pending) | self._wn_done
        if done != set(w.bwd_tables):  # every group's GEMMs ran (their slabs are final)
            raise RuntimeError(f"batched weight-norm backward: groups {set(w.bwd_tables) - done} did not run")
        self._wn_run(w)

    def _blk(self, w, side, si, j, kind, l):
        """Partial-sum buffer `kind` of layer l of block j (encoder / decoder
        stage si): the block's own when the weight-norm backward is batched,
        else the workspace's shared one."""
        parts = w.blk_parts.get((side, si, j))
        return parts[kind][l] if parts is not None else getattr(w, kind)[l]

    def _gnb(self, w, si, j):
        """GNBWD epilogue arguments: the GEMM producing dL/dc_{j+1} of encoder
        stage si also writes block j's (last layer's) GroupNorm-backward sums."""
        sw = w.enc[si]
        if not sw.fuse:
            return {}
        gn = self.enc_stages[si].blocks[j].gns[-1]
        return dict(gn_bwd=w.gnb_part_enc, gn_h=sw.h[j][-1], gn_mr=sw.mr[j][-1], gn_gamma=gn.weight, gn_beta=gn.bias,
                    gn_groups=1)

    @staticmethod
    def _gnb_parts(sw, cols, fused=True):
        """GNBWD tiles per utterance (0 = vqx_gn_bwd reduces itself)."""
        return (sw.T // 128) * ((cols + 127) // 128) if (sw.fuse and fused) else 0

    @staticmethod
    def _bview(buf, B, C):
        return buf.view(-1)[: B * C].view(B, C)

    def _enc_cur(self, w, si, k):
        sw = w.enc[si]
        return Workspace.view(w.dc_flat[k], sw.N, sw.C)

    def _producer_into_enc(self, w, si, dst, colsum_buf, gnb_ok):
        """Epilogue kwargs for a dgrad whose output is dL/dc_nb of encoder stage si
        (its last block's input gradient): bias partials and, when the stage's
        last block exists and the producer is unfolded, its GNBWD sums."""
        kw = dict(colsum=colsum_buf)
        st = self.enc_stages[si]
        if st.blocks and gnb_ok:
            kw.update(self._gnb(w, si, len(st.blocks) - 1))
        return kw

    def encoder_bwd(self, w, grad_scale=1.0, dz=None):
        """Backward of beta*z_enc_loss through the encoder: the commitment term is
        the encoder's only gradient source (z_vq is a no-grad gather under
        reduction='frame_mean', layers_vq.py:292,315).  `dz` (frame-major
        [B*T_z, Z] f32) replaces that source: parity tests feed the same
        well-conditioned dL/dz to this path and to autograd of the oracle."""
        B = w.B
        # the encoder output conv's bias gradient: column sums of dL/dz into the rows of
        # w.cs_eo, added by the "enc_out" group's weight-norm backward
        if dz is None and not self.plain:  # EMA: the commitment term is the encoder's only gradient
            ops.vq_commit_bwd_cs(w.z, w.zq, 2.0 * self.m.beta * grad_scale / w.Nz, w.dz, w.cs_eo)
            w.cs_eo_full = True  # every row written (allocated zero: the other path needs no clear until then)
        else:
            if dz is not None:
                ops.convert_2d(dz, w.dz)
            self.bias_grad(w.cs_eo, w.dz, zero_tail=getattr(w, "cs_eo_full", False))
            w.cs_eo_full = False
        eo = self.enc_out
        ne = len(self.enc_stages)
        last = w.enc[-1]
        k = 0
        cur = self._enc_cur(w, ne - 1, k)
        self.wgrad_dgrad(eo, w.dz, last.a[-1], cur, last.T, mask=last.a[-1], mask_slope=0.2,
                         **self._producer_into_enc(w, ne - 1, None, last.cs[-1], True))
        self._wn_bwd(w, "enc_out")
        for si in reversed(range(ne)):
            st, sw = self.enc_stages[si], w.enc[si]
            T, N, C = sw.T, sw.N, sw.C
            dh = Workspace.view(w.dh_flat, N, C)
            tmp = Workspace.view(w.tmp_flat, N, C)
            dy2 = Workspace.view(w.dy_flat, N, C)
            nb = len(st.blocks)
            # the producer of dL/dc_nb (output conv or next stage conv) fused GNBWD only when unfolded
            top_fused = si == ne - 1 or self.enc_stages[si + 1].conv.kind != KIND_DOWN
            for j in reversed(range(nb)):
                b = st.blocks[j]
                k ^= 1
                nxt = self._enc_cur(w, si, k)
                # cur = dL/dc_{j+1}, the gradient w.r.t. block j's output GN(h_L) + skip(c_j)
                dy = cur
                fused_here = top_fused if j == nb - 1 else True
                for l in reversed(range(st.L)):
                    Lr, gn = b.convs[l], b.gns[l]
                    cs_b = self._bview(self._blk(w, "enc", si, j, "colsum_b", l), B, C)
                    dg_b = self._bview(self._blk(w, "enc", si, j, "dgam_b", l), B, C)
                    db_b = self._bview(self._blk(w, "enc", si, j, "dbet_b", l), B, C)
                    nparts = self._gnb_parts(sw, C, fused_here) if l == st.L - 1 else 0
                    ops.gn_bwd(dy, sw.h[j][l], dh, T, 1, False, sw.mr[j][l], gn.weight, gn.bias, w.gnb_part_enc,
                               cs_b, dg_b, db_b, nparts=nparts)
                    src = sw.a[j] if l == 0 else sw.g[j][l - 1]
                    if l > 0:  # into LeakyReLU(GN(h_{l-1})): its derivative from the sign of the stored output
                        self.wgrad_dgrad(Lr, dh, src, dy2, T, mask=sw.g[j][l - 1], mask_slope=0.2)
                        dy = dy2
                    else:
                        self.wgrad_dgrad(Lr, dh, src, tmp, T, mask=sw.a[j], mask_slope=0.2)
                # the skip conv last, adding the stack's data gradient with the column sums and the
                # previous block's GroupNorm-backward sums in its epilogue.  (Round 4: the skip conv
                # first with a plain epilogue and those reads in the 3-tap DGRAD's epilogue instead
                # measured +10 us per block: the 3-tap DGRAD runs two rounds of workgroups and pays
                # the epilogue twice, profiles/r04/enc_bwd_order.txt.)
                prod = dict(colsum=sw.cs[j])
                if j > 0:
                    prod.update(self._gnb(w, si, j - 1))
                self.wgrad_dgrad(b.skip, cur, sw.c[j], nxt, T, res=tmp, **prod)
                # weight norms of the stack convs and skip + their biases and the GN affine
                self._wn_bwd(w, b.key)
                cur = nxt
            # cur = dL/dc_0 of the stage (the stage conv's output)
            if si == 0:  # the mel batch needs no gradient
                self.wgrad(st.conv, cur, w.x, T)
            else:
                prev = w.enc[si - 1]
                self.wgrad(st.conv, cur, prev.a[-1], T)
                k ^= 1
                pcur = self._enc_cur(w, si - 1, k)
                if st.conv.kind == KIND_DOWN:  # folded: no column epilogues, colsum separately
                    self.dgrad(st.conv, cur, pcur, T, mask=prev.a[-1], mask_slope=0.2)
                    ops.colsum(pcur, w.cs_part_enc, prev.cs[-1][0])
                else:
                    self.dgrad(st.conv, cur, pcur, T, mask=prev.a[-1], mask_slope=0.2,
                               **self._producer_into_enc(w, si - 1, None, prev.cs[-1], True))
                cur = pcur
            self._wn_bwd(w, ("enc_stage", si))

    def _dec_dr(self, w, si, k):
        return w.dec[si].dr[k]

    def decoder_bwd(self, w):
        B, S = w.B, self.dims["S"]
        f1, f2 = self.fin1, self.fin2
        dxhat = w.dxhat
        ns = len(self.dec_stages)
        self.bias_grad(w.cs_f2, dxhat)
        if self.fin2_pad is not None:
            Fp, wfull = self.fin2_pad
            pol = self.opt.kernel_policy
            ops.conv_dgrad_wgrad(w.dxhat_pad, wfull, w.df1,
                                 dict(T=w.T, cin=Fp, cout=f2.cin, ntaps=1, pad=0, dil=1, policy=pol, mask=w.f1,
                                      mask_slope=0.0, colsum=w.cs_f1),
                                 dxhat, w.f1, f2.slab, dict(T=w.T, ntaps=1, pad=0, dil=1, splits=f2.splits, policy=pol,
                                                            r_dim=f2.cout, c_dim=f2.cin, shift_sign=1))
        else:
            self.wgrad_dgrad(f2, dxhat, w.f1, w.df1, w.T, mask=w.f1, mask_slope=0.0, colsum=w.cs_f1)
        s = math.sqrt(1.0 / self.n_dec_layers)
        # dL/dskip (identical for every block) -> tail columns of every [dx | dskip] buffer
        lst = ns - 1
        sw = w.dec[lst]
        k = 0
        cur = sw.dr[k]
        self.wgrad_dgrad(f1, w.df1, w.a_skip, cur[:, sw.C:], w.T, mask=w.a_skip, mask_slope=0.0, mask_scale=s,
                         colsum=w.cs_skip)
        targets = [w.dec[si].dr[q][:, w.dec[si].C:] for si in range(ns) if self.dec_stages[si].blocks
                   for q in range(2) if not (si == lst and q == k)]
        if len(targets) == 1:
            # the copy and the zero dL/dx at the decoder output (the last residual is unused) in one pass
            ops.convert_2d_zero2(cur[:, sw.C:], targets[0], cur[:, :sw.C])
        else:
            for t in targets:
                ops.convert_2d(cur[:, sw.C:], t)
            ops.convert_2d(None, cur, cols=sw.C)  # dL/dx at the decoder output is 0: the last residual is unused
        # (its bias-gradient partials sw.cs[-1] are zero since the workspace was allocated)
        self._wn_bwd(w, "fin")
        cur_x = cur[:, :sw.C]
        for si in reversed(range(ns)):
            st, sw = self.dec_stages[si], w.dec[si]
            T, C = sw.T, sw.C
            C2 = 2 * C
            dg = Workspace.view(w.dg_flat, sw.N, C)
            du = Workspace.view(w.du_flat, sw.N, C2)
            for j in reversed(range(len(st.blocks))):
                b = st.blocks[j]
                dg_b = self._bview(self._blk(w, "dec", si, j, "dgam_b", 0), B, C2)
                db_b = self._bview(self._blk(w, "dec", si, j, "dbet_b", 0), B, C2)
                ci, gn, rs = b.conv_in, b.gn, b.rs
                nxt = sw.dr[k ^ 1]
                # cur = [dL/dx_{j+1} | dL/dskip]
                # (sw.fuse: GLU + GroupNorm backward sums from the res/skip dgrad's epilogue)
                gkw = dict(gn_bwd=w.gnb_part, gn_h=sw.u[j], gn_mr=sw.mr[j], gn_gamma=gn.weight, gn_beta=gn.bias,
                           gn_groups=2, gn_glu=True) if sw.fuse else {}
                self.wgrad_dgrad(rs, cur, sw.g[j], dg, T, **gkw)
                ops.gn_bwd(dg, sw.u[j], du, T, 2, True, sw.mr[j], gn.weight, gn.bias, w.gnb_part, sw.cs_all[j],
                           dg_b, db_b, nparts=self._gnb_parts(sw, C))
                self.wgrad_dgrad(ci, du, sw.xs[j], nxt[:, :C], T, res=cur[:, :C], colsum=sw.cs[j])
                # weight norms of conv_in/res_skip + biases of res_skip, conv_in and the GN affine
                self._wn_bwd(w, b.key)
                k ^= 1
                cur = nxt
                cur_x = cur[:, :C]
            # cur_x = dL/dx_0 of the stage (the stage conv's output)
            if st.conv.kind == KIND_UP and not cur_x.is_contiguous():  # the folded GEMMs need whole rows
                ops.convert_2d(cur_x, dg)
                cur_x = dg
            if si > 0:
                prev, pst = w.dec[si - 1], self.dec_stages[si - 1]
                self.wgrad(st.conv, cur_x, prev.xs[-1], T)
                if pst.blocks:
                    k = 0
                    pcur = prev.dr[k]
                    dst = pcur[:, :prev.C]
                else:
                    pcur = None
                    dst = prev.dx
                if st.conv.kind == KIND_UP:
                    self.dgrad(st.conv, cur_x, dst, T)
                    ops.colsum(dst, w.cs_part, prev.cs[-1][0])
                else:
                    self.dgrad(st.conv, cur_x, dst, T, colsum=prev.cs[-1])
                self._wn_bwd(w, ("dec_stage", si))
                cur, cur_x = pcur, dst
            else:
                self.wgrad(st.conv, cur_x, w.zq_in, T)
                if self.plain:  # straight-through VQ: the decoder input's gradient reaches the encoder
                    self.dgrad(st.conv, cur_x, w.dzq, T)
                self._wn_bwd(w, ("dec_stage", 0))
        # speaker conditioning of all blocks: dW, bias and d(embedding), per output width
        emb_g = self.g(self.m.embeds._embedding.weight)
        if not self.cond_groups:  # the embedding feeds nothing: its gradient is zero
            ops.zero_(emb_g)
        for gi, (O, blocks) in enumerate(self.cond_groups.items()):
            if getattr(w, "cond_ids_mode", False):
                ops.linear_batched_bwd_ids(w.cond_tables[O], self.m.embeds._embedding.weight, w.y_dev, B,
                                           blocks[0].cond.cin, O, w.dyemb, w.lin_part)
            else:
                ops.linear_batched_bwd(w.cond_tables[O], w.yemb, B, blocks[0].cond.cin, O, w.dyemb, w.lin_part)
            ops.embedding_bwd_rows(w.dyemb, w.y_dev, emb_g, accumulate=gi > 0)  # every row written: no zero fill
        self._wn_bwd_cond(w)

    def _wn_bwd_cond(self, w):
        self._wn_bwd(w, "cond")

    # ------------------------------------------------------------ quantizer
    def vq_init_if_needed(self, w):
        """init_emb (layers_vq.py:192-201) on the first training forward."""
        q = self.m.quantizer
        if q.initialized:
            return False
        K = self.dims["K"]
        if w.Nz * self.world < K:  # N_global < K: noisy tiling of the global batch (identical on every rank)
            rows = self._tile_rows(w)
            q.embeddings.copy_(rows)
        else:
            perm = self._perm_rows(w.Nz * self.world, K, self.rank * w.Nz, w.Nz if self.comm is not None else None)
            ops.gather_rows_host(w.z, perm, q.embeddings)
            if self.comm is not None:
                self.comm.all_reduce_sum(q.embeddings)
        ops.convert_2d(q.embeddings, q.emb_sum)
        q.emb_elem.fill_(1.0)
        q.mark_initialized()
        return True

    def vq_plain_forward(self, w):
        """VectorQuantizer.forward (layers_vq.py:79-150): renormalise the
        codebook parameter in place and the frames, nearest code, per-code
        sums / counts (for the codebook gradient) and the perplexity."""
        q = self.m.quantizer
        ops.zero_(w.ema)
        if self.vq_normalize:
            ops.vq_normalize(w.z, q.embeddings.data, w.z_norm, w.z_len, w.embn, w.e_len, w.pv_part, w.stats[2:3])
            zin, emb = w.z_norm, w.embn
        else:
            zin, emb = w.z, q.embeddings.data
        ops.vq_forward(zin, emb, w.idx, w.zq, w.zq_c, w.stats[1:2], w.vq_part, w.bsum, w.bcnt)
        ops.vq_perplexity(w.bcnt, w.Nz, w.stats[4:5])

    def vq_plain_backward(self, w):
        """Straight-through + codebook + commitment (+ normalisation) gradients."""
        q = self.m.quantizer
        zin = w.z_norm if self.vq_normalize else w.z
        emb = w.embn if self.vq_normalize else q.embeddings.data
        ops.vq_plain_bwd(w.z, zin, w.z_len if self.vq_normalize else None, w.zq, w.dzq,
                         w.src_t if w.jittered else None, w.Tz, self.vq_normalize, float(self.m.beta), 2.0 / w.Nz,
                         w.dz, w.bsum, w.bcnt, emb, w.e_len if self.vq_normalize else None, self.g(q.embeddings))

    def vq_forward_train(self, w, defer_stats=False):
        """defer_stats: the EMA statistics are left to the second stream
        (_enc_bwd_early runs them there before the encoder backward)."""
        w.stats_deferred = False
        if self.plain:
            return self.vq_plain_forward(w)
        q = self.m.quantizer
        K = self.dims["K"]
        self.vq_init_if_needed(w)
        w.ev_ema = None
        if self._side_on:
            # distance/argmin/gather on the GEMM chain; the EMA statistics and the
            # codebook update (update_emb, layers_vq.py:203-233) on the side stream:
            # only the next step's distance kernel reads their results
            ops.vq_forward(w.z, q.embeddings, w.idx, w.zq, w.zq_c, w.stats[1:2], w.vq_part, None, None)
            side = self._fork()
            with torch.cuda.stream(side):
                ops.zero_(w.ema)
                ops.vq_stats(w.z, w.idx, K, w.vq_part, w.bsum, w.bcnt)
                self._ema_rows(w, K)
                if self.comm is not None:
                    self.comm.all_reduce_sum(w.ema, async_op=True).wait()
                self._ema_apply(w)
            w.ev_ema = side.record_event()
            return
        if not getattr(w, "ema_clean", False):  # bsum / bcnt not left zero by the last update (rand_rows: overwritten)
            ops.zero_(w.ema)
        w.ema_clean = False
        # the commitment partials' sum (stats[1]) is left to the log-loss launch (train_forward)
        if defer_stats:
            ops.vq_forward(w.z, q.embeddings, w.idx, w.zq, w.zq_c, None, w.vq_part, None, None)
            w.stats_deferred = True
        else:
            ops.vq_forward(w.z, q.embeddings, w.idx, w.zq, w.zq_c, None, w.vq_part, w.bsum, w.bcnt)
        w.vq_sum_pending = (w.Nz + ops.VQ_FRAMES - 1) // ops.VQ_FRAMES
        # one process with the fused close: the rows are read from z inside the EMA launch
        self._ema_rows(w, K, defer=self.opt.fused_close and self.comm is None and K <= 512)
        if self.comm is not None:
            self._ema_work = self.comm.all_reduce_sum(w.ema, async_op=True)

    def _ema_rows(self, w, K, defer=False):
        """rand_rows for dead-code replacement: z[randperm(N)[:K]] (update_emb,
        layers_vq.py:212-213).  defer: the permutation is drawn here (the CPU
        generator's order) and kept in w.ema_perm for the EMA launch to read the
        rows from z itself (vqx_step_close.rows_src)."""
        w.ema_perm = None
        if w.Nz * self.world < K:
            rows = self._tile_rows(w)
            if self.rank != 0:  # every rank holds the same rows; the EMA bundle is SUM-reduced
                rows.zero_()
            w.rand_rows.copy_(rows)
        else:
            perm = self._perm_rows(w.Nz * self.world, K, self.rank * w.Nz, w.Nz if self.comm is not None else None)
            if defer:
                w.ema_perm = perm
                return
            ops.gather_rows_host(w.z, perm, w.rand_rows)

    def _ema_apply(self, w, sums=(), publish=None):
        """The EMA update; it leaves bsum / bcnt zero (clear=True), so the next
        step's accumulation needs no zero fill of the statistics."""
        q = self.m.quantizer
        perm = getattr(w, "ema_perm", None)
        res = ops.vq_ema_update(q.emb_sum, q.emb_elem, q.embeddings, w.bsum, w.bcnt, w.rand_rows, q.mu, q.threshold,
                                w.stats[4:8], w.ema_part, clear=True, sums=sums, publish=publish,
                                rows=(w.z, perm) if perm is not None else None)
        w.ema_perm = None
        w.ema_clean = True
        return res

    def vq_ema_update(self, w):
        """End of the step: apply the EMA update (or, when it ran on the side
        stream, order the current stream after it)."""
        if self.plain:  # the straight-through codebook is a parameter updated by Adam
            return
        if getattr(w, "ev_ema", None) is not None:
            torch.cuda.current_stream().wait_event(w.ev_ema)
            w.ev_ema = None
            return
        if getattr(w, "ema_applied", False):  # already run at the end of the forward
            w.ema_applied = False
            return
        self._ema_finish(w)

    def _ema_finish(self, w, sums=(), publish=None):
        """Wait for the EMA bundle's all-reduce (data parallel), then update
        (sums / publish: ops.vq_ema_update's closing work; returns its (seq, slot))."""
        if getattr(self, "_ema_work", None) is not None:
            self.comm.wait(self._ema_work, "ema")
            self._ema_work = None
        if getattr(w, "ev_stats", None) is not None:  # statistics from the second stream (vq_stats_side)
            torch.cuda.current_stream().wait_event(w.ev_stats)
            w.ev_stats = None
        return self._ema_apply(w, sums, publish)

    # ------------------------------------------------------------ full step
    world, rank, comm = 1, 0, None

    def attach_comm(self, comm):
        """Run the data-parallel path over `comm` (parallel/ddp.py Comm): the
        per-group gradient mean all-reduces, the EMA-statistics sum and the
        owned-rows assembly of the dead-code rows.  The Trainer attaches one
        when the process group has more than one rank; tests attach a
        world-size-1 group to run the RCCL branch on one GPU, where every
        collective is the identity and the step must equal the plain one."""
        self.world, self.rank, self.comm = comm.world, comm.rank, comm

    def forward_train(self, x, y, early_bwd=False):
        """Training forward (saves every activation the backward needs).
        x (B, mel, T) f32 device, y (B, 1) int64 device."""
        B, _, T = x.shape
        self._join()
        w = self.ws(B, T, train=True)
        w.y_dev = y.reshape(-1)
        w.x_nct = x
        w.ev_cond = None
        fused = self._fused_prologue(w, x)
        if not fused:
            self.pack_weights()
            if self._side_on:  # the conditioning row biases are first read by the decoder
                side = self._fork()
                with torch.cuda.stream(side):
                    self.embed_and_cond(w, w.y_dev)
                w.ev_cond = side.record_event()
            else:
                self.embed_and_cond(w, w.y_dev)
        self.encoder_fwd(w, x, transposed=fused)
        early = early_bwd and self.opt.enc_bwd_early and self._bwd_concurrent()
        self.vq_forward_train(w, defer_stats=early and self.opt.vq_stats_side and not self._side_on)
        if early:
            self._enc_bwd_early(w)
        w.zq_in = w.zq_c
        w.jittered = False
        if self.dims["jitter_p"] > 0 and self.m.jitter.training:
            src = torch.from_numpy(self.jitter_map(w.Tz)).pin_memory()
            w.src_t.copy_(src, non_blocking=True)
            ops.time_gather(w.zq_c, w.zq_j, B, w.Tz, w.src_t)
            w.zq_in = w.zq_j
            w.jittered = True
        if w.ev_cond is not None:
            torch.cuda.current_stream().wait_event(w.ev_cond)
        self.decoder_fwd(w, w.zq_in)
        n_vq = getattr(w, "vq_sum_pending", 0)
        close = self.opt.fused_close and not self._side_on and not self.plain
        sums = ()
        if close:
            # the log-loss partials (and the VQ commitment partials) summed in the
            # EMA update's last workgroup (vqx_vq_ema_update_close), as the
            # log-loss's final launch would: the same scale, in float32
            n_l = ops.logloss_parts(x, w.xhat, 1.0 / (B * T), w.dxhat, w.loss_part)
            sums = [(w.loss_part[:n_l], float(np.float32(1.0) / (np.float32(B) * np.float32(T))), w.stats[0:1])]
            if n_vq:
                sums.append((w.vq_part[:n_vq], 1.0, w.stats[1:2]))
            w.vq_sum_pending = 0
        elif n_vq:  # the VQ commitment partials summed in the log-loss's final launch
            ops.logloss_fwd_bwd_x(x, w.xhat, 1.0 / (B * T), w.dxhat, w.stats[0:1], w.loss_part, w.vq_part[:n_vq],
                                  w.stats[1:2])
            w.vq_sum_pending = 0
        else:
            ops.logloss_fwd_bwd(x, w.xhat, 1.0 / (B * T), w.dxhat, w.stats[0:1], w.loss_part)
        # Round 6: the EMA codebook update here, where the reference runs it
        # (inside the forward, layers_vq.py:295-296; the backward reads no
        # codebook in EMA mode), so every loss statistic is final at the end of
        # the forward: snapshot them and mark the point with an event
        # (trainer/basic.py LazyLossDetail reads them without waiting for the
        # backward).  The side-stream schedule keeps its end-of-step join.
        w.stats_snap = None
        if not self._side_on:
            publish = self.opt.lazy_stats and self.opt.early_stats
            if publish:
                # published into a host mailbox (ops.Mailbox): the host polls a
                # sequence number, so no event marker enters the stream (a
                # recorded event idled it ~6 us at every step)
                if self._mailbox is None:
                    self._mailbox = ops.Mailbox(64, 16)
                snap = torch.empty_like(w.stats)  # the device copy, for reads after the slot was reused
            pub_stream = torch.cuda.current_stream()
            if close:  # the sums and the publish in the EMA update's last workgroup
                seq, slot = self._ema_finish(w, sums=sums, publish=(self._mailbox, w.stats, snap) if publish else None) \
                    or (None, None)
                w.ema_applied = True
            else:
                if not self.plain:
                    self._ema_finish(w)
                    w.ema_applied = True
                if publish:
                    seq, slot = self._mailbox.publish(w.stats, snap)  # vqx_mailbox_publish
            if publish:
                w.stats_snap = (self._mailbox, seq, slot, snap, pub_stream)
        return w


    def _bwd_begin(self, w):
        """The backward's bookkeeping (weight-norm groups, gradient-norm partials,
        split-K reduction layers)."""
        if self.comm is not None:
            self._grads_reset()
        self._wn_pending, self._wn_done = [], set()
        self._sq_plan_ready = None
        self._sq_off, self._sq_runs = 0, []
        self._wn_active = True
        if self.comm is None and self.opt.fuse_grad_norm and self._wn_batched():
            self._sq_buf(w)  # allocated before any second stream runs
        self._fix_now = getattr(w, "fix", frozenset())

    def _enc_bwd_early(self, w):
        """EngineOptions.enc_bwd_early: the encoder backward issued on the second
        stream right after the VQ forward, beside the decoder forward (it needs
        only z, the gathered codes and the encoder's activations)."""
        self._bwd_begin(w)
        side = self._fork()
        w.ev_stats = None
        with torch.cuda.stream(side):
            if getattr(w, "stats_deferred", False):  # the EMA statistics first; the EMA update waits for them
                ops.vq_stats(w.z, w.idx, self.dims["K"], w.vq_part, w.bsum, w.bcnt)
                w.ev_stats = side.record_event()
                w.stats_deferred = False
            self.encoder_bwd(w)
            self._wn_enc_run(w, concurrent=True)
        w.enc_bwd_early = True

    def _wn_enc_run(self, w, concurrent=False):
        """After the encoder backward (on its stream under bwd_streams).  One
        process: the encoder groups' batched weight-norm backward as a launch of
        its own (wn_bwd_split), the decoder groups' at the end.  Data parallel on
        two streams: the encoder's pending groups, and every gradient run then
        final, leave from the encoder's stream -- an all-reduce waits for the
        stream it is issued from, so no run may mix the two chains' gradients
        (the decoder's are not final yet: its backward is issued after)."""
        if not self._wn_batched():
            return
        if self.comm is not None:
            if concurrent:
                self._wn_run(w)
                self._grads_final([], flush=True)
        elif self.opt.wn_bwd_split:
            self._wn_run(w)

    def _bwd_concurrent(self):
        """EngineOptions.bwd_streams applies: EMA quantizer, batched weight-norm
        backward; data parallel with bwd_streams_ddp (the encoder's gradient
        runs all-reduced from its stream, _wn_enc_run)."""
        return (self.opt.bwd_streams and self.device.type == "cuda" and not self.plain and self.opt.wn_bwd_batch
                and (self.comm is None or self.opt.bwd_streams_ddp))

    def backward(self, w, grad_loss=None):
        """Data parallel: every backward group's gradients are all-reduced as
        soon as its weight-norm backward has finalised them (_wn_bwd), so the
        reduces overlap the rest of the backward; the remainder (embedding,
        codebook) is flushed at the end."""
        early = getattr(w, "enc_bwd_early", False)
        w.enc_bwd_early = False
        if not early:
            self._bwd_begin(w)
        try:
            if early:
                # the encoder backward is already on the second stream (forward_train)
                self.decoder_bwd(w)
                self._join()
            elif self.plain:
                # straight-through: the encoder's gradient comes through the decoder
                self.decoder_bwd(w)
                self.vq_plain_backward(w)
                self.encoder_bwd(w)
            elif self._bwd_concurrent():
                # the encoder backward on a second stream beside the decoder's: the
                # decoder input carries no gradient (z_vq is a no-grad gather,
                # layers_vq.py:292,315), so the two chains share no data; the
                # encoder's scratch is its own (gnb_part_enc, cs_part_enc) and every
                # group's split-K slabs and column partials have their own region
                # (wn_bwd_batch)
                # the encoder groups' weight-norm backward follows them there
                side = self._fork()
                with torch.cuda.stream(side):
                    self.encoder_bwd(w)
                    self._wn_enc_run(w, concurrent=True)
                self.decoder_bwd(w)
                self._join()
            else:
                self.encoder_bwd(w)
                self._wn_enc_run(w)
                self.decoder_bwd(w)
            self._wn_bwd_flush(w)
            self._sq_finish(w)
        finally:
            self._wn_active = False
            self._fix_now = frozenset()
        if self.comm is not None:
            self._grads_final(range(len(self.params)), flush=True)
            self.comm.finish()

    def init_optimizer(self, lr, betas=(0.5, 0.999), eps=1e-8, max_grad_norm=10.0, sched_step=None, sched_gamma=1.0,
                       kind="adam"):
        """kind 'adam' (torch.optim.Adam, trainer/basic.py:36-39) or 'radam'
        (trainer/radam.py RAdam, basic.py:30-34); both fused with the
        global-norm clip and StepLR."""
        if kind not in ("adam", "radam"):
            raise ValueError(f"unknown optimizer {kind!r}")
        self.opt_kind = kind
        dev = self.device
        self.exp_avg = self._zeros(self.n_params, dtype=F32)
        self.exp_avg_sq = self._zeros(self.n_params, dtype=F32)
        self.opt_step = self._zeros(1, dtype=torch.int64)
        self.hyper = self._zeros(16, dtype=F32)
        self.sumsq = self._zeros(1, dtype=F32)
        self.norm_part = self._zeros(1024, dtype=F32)
        self.lr0, self.betas, self.eps, self.max_grad_norm = lr, betas, eps, max_grad_norm
        self.sched_step = sched_step or (1 << 30)
        self.sched_gamma = sched_gamma
        self.opt_ready = True

    def optimizer_step(self):
        plan, self._sq_plan_ready = self._sq_plan_ready, None
        hyper_done = False
        if self.max_grad_norm > 0:
            if plan is not None and self.opt_kind != "radam":  # + Adam's per-step scalars in the same launch
                ops.sq_norm_finish_adam(plan[0], self.flat_g, plan[1], self.sumsq, self.norm_part, self.opt_step,
                                        self.lr0, self.sched_gamma, self.sched_step, self.betas[0], self.betas[1],
                                        self.eps, self.hyper)
                hyper_done = True
            elif plan is not None:  # partials from this step's weight-norm backward
                ops.sq_norm_finish(plan[0], self.flat_g, plan[1], self.sumsq, self.norm_part)
            else:
                ops.grad_sq_norm(self.flat_g, self.norm_part, self.sumsq)
        sumsq = self.sumsq if self.max_grad_norm > 0 else None
        if self.opt_kind == "radam":
            ops.radam_hyper(self.opt_step, self.lr0, self.sched_gamma, self.sched_step, self.betas[0], self.betas[1],
                            self.eps, self.hyper)
            ops.radam_step(self.flat_p, self.flat_g, self.exp_avg, self.exp_avg_sq, self.hyper, sumsq,
                           float(self.max_grad_norm))
            return
        if not hyper_done:
            ops.adam_hyper(self.opt_step, self.lr0, self.sched_gamma, self.sched_step, self.betas[0], self.betas[1],
                           self.eps, self.hyper)
        if not self._adam_wn_built:
            self._adam_wn = self._adam_wn_plan() if self.opt.fuse_adam_wn else None
            self._adam_wn_built = True
        if self._adam_wn is not None:
            rows, segs = self._adam_wn[0], self._adam_wn[1]
            ops.adam_step_wn(self.flat_p, self.flat_g, self.exp_avg, self.exp_avg_sq, self.hyper, sumsq,
                             float(self.max_grad_norm), rows, segs)
            self._packed_version = self._param_version()
            return
        ops.adam_step(self.flat_p, self.flat_g, self.exp_avg, self.exp_avg_sq, self.hyper, sumsq,
                      float(self.max_grad_norm))

    def _param_version(self):
        """Sum of the version counters of flat_p and of every parameter: any
        in-place torch op on them (copy_, mul_, load_state_dict, a broadcast)
        changes it; the HIP kernels' writes do not.  Edits through `.data`
        bypass version counters: call invalidate_packed() after those."""
        return self.flat_p._version + sum(p._version for p in self.params)

    def invalidate_packed(self):
        """The next forward packs every layer from the parameters (fuse_adam_wn).
        Called by Model.load_state_dict and after the Trainer's initial
        broadcast; any other write to the parameters that bypasses torch's
        version counters (.data, raw kernels, collectives) must call it too --
        EngineOptions.debug_checks verifies it at every forward."""
        self._packed_version = None

    def _check_packed(self):
        """debug_checks: the packed weights and row norms the fused Adam left
        equal a full weight-norm pack of the current parameters."""
        before = [(Lr.wp.clone(), Lr.norm.clone()) for Lr in self.convs]
        ops.weight_norm_fwd(self.wn_fwd_table)
        for Lr, (wp, nm) in zip(self.convs, before):
            if not (torch.equal(wp, Lr.wp) and torch.equal(nm, Lr.norm)):
                raise RuntimeError(f"{Lr.name}: packed weights are stale (parameters written without "
                                   "invalidate_packed())")

    def _adam_wn_plan(self):
        """(rows table, flat segments, forward table of what is left to pack,
        its flags) for vqx_adam_step_wn, or None when the model has nothing it
        can take.  Rows: the weight-normed Conv1d (kind 0) and, when every one
        of them qualifies, ConvTranspose (kind 1) layers whose rows fit the
        kernel's partitions (include/vqx.h)."""
        base, esz = self.flat_p.data_ptr(), (2 if self.cd == torch.bfloat16 else 4)
        ents = [self._wn_entry(Lr, bwd=False) for Lr in self.convs]

        def ok(e):
            if e["g"] is None or e["kind"] not in (0, 1):
                return False
            vo = (e["v"].data_ptr() - base) // 4
            if vo % 4 or (e["v"].data_ptr() - base) % 4:
                return False
            if e["kind"] == 1:
                return (e["cout"] * e["k"]) % 4 == 0 and e["cout"] * e["k"] <= 4096
            cols = e["cin"] * e["k"]
            if cols % 4:
                return False
            if e["k"] > 1:
                return cols <= 4096
            return e["cin"] <= 512 and (e["cin"] * esz) % 16 == 0 and e["w_packed"].data_ptr() % 16 == 0

        conv0 = [e for e in ents if e["kind"] == 0 and ok(e)]
        convt = [e for e in ents if e["kind"] == 1]
        convt = convt if convt and all(ok(e) for e in convt) else []
        rows = conv0 + convt
        if not rows or len(rows) > 128:
            return None
        iv = []
        for e in rows:
            for t in (e["v"], e["g"]):
                lo = (t.data_ptr() - base) // 4
                iv.append((lo, lo + t.numel()))
        iv.sort()
        segs, cur = [], 0
        for lo, hi in iv:
            if lo < cur:
                return None
            if lo > cur:
                segs.append((cur, lo - cur))
            cur = hi
        if cur < self.n_params:
            segs.append((cur, self.n_params - cur))
        if len(segs) > 128:
            return None
        packed = {id(e["w_packed"]) for e in conv0}
        rest = [e for e in ents if id(e["w_packed"]) not in packed]
        sh = torch.tensor(segs, dtype=torch.int64).view(-1, 2)
        sd = sh.to(self.device) if segs else sh
        flags = ops.WNF_NORMS_READY if convt else 0
        return ops.wn_table(rows), (sh, sd), (ops.wn_table(rest) if rest else None), flags

    def train_step(self, x, y):
        """One full training step (trainer/basic.py:55-79): forward, backward,
        clip, Adam, StepLR, EMA codebook update.  Returns the device stats
        vector [x_loss, sqerr, -, -, entropy, used_curr, usage, diff_emb]."""
        if not self.opt_ready:
            raise RuntimeError("init_optimizer() first")
        w = self.forward_train(x, y, early_bwd=True)  # this step's backward follows at unit loss scale
        self.backward(w)
        self.optimizer_step()
        self.vq_ema_update(w)
        return w

    def total_loss(self, w):
        """(total, VQ loss) device scalars of the step's loss (vqvae.py:83)."""
        n = w.Nz
        xl = w.stats[0:1]
        if self.plain:
            qut = w.stats[1:2] / n
            enc = (w.stats[1:2] + w.stats[2:3]) / n
            return (xl + qut) + self.m.beta * enc, enc
        vq = w.stats[1:2] / n
        return xl + self.m.beta * vq, vq

    def loss_detail(self, w, stats_host):
        """The reference's loss dict (vqvae.py:85-87, layers_vq.py:228-233 / 112-116)."""
        s = stats_host.tolist()
        n = w.Nz
        if self.plain:
            f = np.float32
            qut, enc, xl = f(s[1]) / f(n), (f(s[1]) + f(s[2])) / f(n), f(s[0])
            return {"Total": float((xl + qut) + f(self.m.beta) * enc), "VQ loss": float(enc), "X like": float(xl),
                    "entropy": s[4]}
        vq = s[1] / n
        xl = s[0]
        d = {"Total": float(np.float32(xl) + np.float32(self.m.beta) * np.float32(vq)), "VQ loss": vq, "X like": xl}
        d.update({"entropy": s[4], "used_curr": s[5], "usage": s[6], "diff_emb": s[7]})
        return d

    # ------------------------------------------------------------ inference
    def _eval_ws(self, B, T):
        return self.ws(B, T, train=False) if (B, T, True) not in self._ws else self._ws[(B, T, True)]

    def forward_eval(self, x, y):
        """model.eval() forward: no EMA init/update, no jitter (layers_vq.py:282,295,354)."""
        B, _, T = x.shape
        self._join()
        w = self._eval_ws(B, T)
        w.y_dev = y.reshape(-1)
        self.pack_weights()
        self.embed_and_cond(w, w.y_dev)
        self.encoder_fwd(w, x)
        q = self.m.quantizer
        if self.plain:  # VectorQuantizer.forward renormalises in eval too (layers_vq.py:95-101)
            self.vq_plain_forward(w)
        else:
            ops.vq_forward(w.z, q.embeddings, w.idx, w.zq, w.zq_c, w.stats[1:2], w.vq_part, None, None)
        w.zq_in = w.zq_c
        self.decoder_fwd(w, w.zq_c)
        ops.logloss_fwd_bwd(x, w.xhat, 1.0 / (B * T), None, w.stats[0:1], w.loss_part)
        ops.ntc_to_nct(w.xhat, w.xhat_nct)
        return w

    def encode(self, x):
        """Model.encode (vqvae.py:45-52): encoder + nearest-code index, (B, T_z) int64."""
        B, _, T = x.shape
        self._join()
        w = self._eval_ws(B, T)
        self.pack_weights()
        self.encoder_fwd(w, x)
        q = self.m.quantizer
        if self.plain:
            return q.encode(w.z.view(B, w.Tz, -1), time_last=False)
        ops.vq_forward(w.z, q.embeddings, w.idx, None, None, None, w.vq_part, None, None)
        return w.idx.view(B, w.Tz).clone()

    def decode(self, z_idx, y):
        """Model.decode (vqvae.py:55-60): codebook gather + decoder, (B, F, T) f32."""
        B, Tz = z_idx.shape
        T = Tz
        for st in self.enc_stages:
            T *= st.scale
        self._join()
        w = self._eval_ws(B, T)
        w.y_dev = y.reshape(-1)
        self.pack_weights()
        self.embed_and_cond(w, w.y_dev)
        q = self.m.quantizer
        ops.gather_rows(q._codebook() if self.plain else q.embeddings, z_idx.reshape(-1).contiguous(), w.zq)
        ops.convert_2d(w.zq, w.zq_c)
        self.decoder_fwd(w, w.zq_c)
        ops.ntc_to_nct(w.xhat, w.xhat_nct)
        return w.xhat_nct.clone()
