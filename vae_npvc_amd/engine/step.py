"""The VQ-VAE training step on MI355X: every arithmetic op of the reference's
hot path is a libvqx HIP kernel launched here on
torch's current stream; torch is used only for device memory and streams.

Step anatomy (frame-major activations [N = B*T, C], see include/vqx.h):

  pack     weight norm of all 44 convs -> packed effective weights (1 launch pair)
  encoder  conv0 | 10 x {k3 conv -> GN stats -> 1x1 skip conv with the
           GroupNorm-apply + residual fused in its epilogue} | 1x1 out conv
           (f32 out).  Each GEMM producing c_i also stores LeakyReLU(c_i), so
           no GEMM applies an activation to its staged operands
                                                                 (vqvae.py:185-192)
  vq       fused distance/argmin/gather/commitment/EMA-statistics kernel
                                                                 (layers_vq.py:268-323)
  decoder  ConvT0 | 10 x {ConvT k3 (+ speaker term as a per-utterance row bias)
           -> GN stats -> GN+tanh*sigmoid -> 1x1 res/skip conv with the
           residual add and the skip accumulation split in its epilogue} |
           ReLU(s*skip) -> 1x1 (ReLU epilogue) -> 1x1            (vqvae.py:298-318)
  loss     log-likelihood + its gradient in one pass            (layers.py:283-296)
  backward encoder (driven only by beta*commitment, the reference quirk:
           z_vq carries no gradient, layers_vq.py:315) and decoder: dgrad GEMMs
           with activation-derivative / residual epilogues, wgrad split-K slabs
           reduced by the weight-norm backward, GN backward (2 passes).
  update   global grad norm -> fused clip + Adam (+ StepLR on device); EMA codebook.

The engine owns flat fp32 buffers for parameters, gradients and Adam moments;
model parameters are views into them, so `model.state_dict()` stays the
reference's and the optimizer touches one contiguous buffer.
"""
import math
import os
from dataclasses import dataclass

import numpy as np
import torch

from .. import _lib as L
from .. import ops

F32 = torch.float32


@dataclass
class ConvLayer:
    mod: object          # WNConv1d
    name: str
    kind: int            # 0 Conv1d, 1 ConvTranspose1d
    cin: int             # effective-conv input channels
    cout: int            # effective-conv output channels
    k: int
    pad: int
    wp: torch.Tensor = None     # packed effective weight [cout, k*cin]
    norm: torch.Tensor = None   # ||v_o||
    slab: torch.Tensor = None   # wgrad partials [splits, rows, cols]
    splits: int = 1

    @property
    def rows(self):
        return self.cin if self.kind == 1 else self.cout

    @property
    def cols(self):
        return (self.cout if self.kind == 1 else self.cin) * self.k


class Workspace:
    """All activations / gradients of one (B, T) shape (allocated once)."""

    def __init__(self, eng, B, T, train=True):
        d, cd, dev = eng.dims, eng.cd, eng.device
        N = B * T
        self.B, self.T, self.N = B, T, N
        e = lambda *s, dt=cd: torch.empty(*s, device=dev, dtype=dt)  # noqa: E731
        C, Z, Cd, S, Fo, mel = d["C"], d["Z"], d["Cd"], d["S"], d["F"], d["mel"]
        ns, nd, K, D = d["ns"], d["nd"], d["K"], d["Z"]
        self.x = e(N, mel)
        self.c = [e(N, C) for _ in range(ns + 1)]
        self.a = [e(N, C) for _ in range(ns + 1)]   # LeakyReLU(c_i), written by the producing GEMM (ACT2)
        self.h = [e(N, C) for _ in range(ns)]
        self.enc_mr = e(ns, B, 2, dt=F32)
        self.z = e(N, Z, dt=F32)
        self.idx = torch.empty(N, device=dev, dtype=torch.int64)
        self.zq = e(N, Z, dt=F32)
        self.zq_c = e(N, Z)
        self.zq_j = e(N, Z) if d["jitter_p"] > 0 else None
        self.src_t = torch.empty(T, device=dev, dtype=torch.int32)
        self.jittered = False
        if eng.plain:  # straight-through quantizer: normalised frames / codebook and their norms
            self.z_norm = e(N, Z, dt=F32)
            self.z_len = e(N, dt=F32)
            self.embn = e(K, Z, dt=F32)
            self.e_len = e(K, dt=F32)
            self.pv_part = e(N // 4 + 8, dt=F32)
        self.vq_part = e(ops.vq_workspace(N, K, True), dt=F32)  # VQ partials + EMA-statistics slabs
        # EMA statistics bundle (all-reduced as one buffer in data parallel)
        self.ema = e(K * D + K + K * D, dt=F32)
        self.bsum = self.ema[: K * D].view(K, D)
        self.bcnt = self.ema[K * D: K * D + K]
        self.rand_rows = self.ema[K * D + K:].view(K, D)
        self.ema_part = e((K * D + 1023) // 1024, dt=F32)  # vqx_vq_ema_update workspace
        self.yemb = e(B, d["ydim"], dt=F32)
        self.condbias = e(nd, B, 2 * Cd, dt=F32)
        self.xs = [e(N, Cd) for _ in range(nd + 1)]
        self.u = [e(N, 2 * Cd) for _ in range(nd)]
        self.g = [e(N, Cd) for _ in range(nd)]
        self.dec_mr = e(nd, B, 4, dt=F32)
        self.skip32 = e(N, S, dt=F32)
        self.a_skip = e(N, S)                       # ReLU(sqrt(1/(nd+1)) * skip)
        self.f1 = e(N, S)                           # ReLU(final conv 1 output)
        self.xhat = e(N, Fo, dt=F32)
        self.xhat_nct = e(B, Fo, T, dt=F32)
        # scalars: 0 x_loss, 1 sqerr, 4..7 EMA diagnostics
        self.stats = torch.zeros(8, device=dev, dtype=F32)
        # GroupNorm partials written by GEMM epilogues (GNSTATS / GNBWD tiles:
        # [N/128][column tile][4]) when T and the group widths are multiples of 128
        self.fuse_gn = (T % 128 == 0 and C % 128 == 0 and Cd % 128 == 0
                        and os.environ.get("VQX_FUSE_GN", "1") != "0")
        self.gn_rg = N // 128 if self.fuse_gn else 0
        self.gst = e(max(1, self.gn_rg) * ((max(C, 2 * Cd) + 127) // 128) * 4, dt=F32)
        self.loss_part = e(1024, dt=F32)
        self.gn_part = e(B * 2 * 8 * 3, dt=F32)
        if not train:
            return
        self.dxhat = e(N, Fo)
        self.df1 = e(N, S)
        self.dr = [e(N, Cd + S) for _ in range(2)]
        self.dg = e(N, Cd)
        self.du = e(N, 2 * Cd)
        self.gnb_part = e(max(B * 64 * 2, max(1, self.gn_rg) * ((max(C, Cd) + 127) // 128) * 4), dt=F32)
        self.colsum_b = e(B * 2 * max(Cd, C), dt=F32)   # per-utterance column sums of du
        self.dgam_b = e(B * 2 * max(Cd, C), dt=F32)
        self.dbet_b = e(B * 2 * max(Cd, C), dt=F32)
        self.dz = e(N, Z)
        self.dzq = e(N, Z) if eng.plain else None  # decoder gradient w.r.t. its (jittered) input
        self.dc = [e(N, C) for _ in range(2)]
        self.dh = e(N, C)
        self.tmp = e(N, C)
        self.dyemb = e(B, d["ydim"], dt=F32)
        self.cs_part = e(64 * max(C, 2 * Cd, Cd + S, mel, 1024), dt=F32)
        # bias-gradient partials: GEMM COLSUM epilogues write [row tile][C]
        # sums of the gradient they produce; the group's weight-norm backward
        # launch reduces them (VQX_WN_COLREDUCE entries)
        tm = (N + L.CONV_TILE_ROWS - 1) // L.CONV_TILE_ROWS
        self.cs_enc = [e(tm, C, dt=F32) for _ in range(2)]   # dL/dc_i (ping-pong)
        self.cs_dec = [e(tm, Cd, dt=F32) for _ in range(2)]  # dL/dx_i (ping-pong)
        self.cs_skip = e(tm, S, dt=F32)                      # dL/dskip
        self.cs_f1 = e(tm, S, dt=F32)                        # dL/d(final conv 1 output)
        # per-utterance column sums of du per decoder block: conv_in and
        # conv_cond bias gradients, and dout of the batched conditioning backward
        self.cs_all = e(nd, B, 2 * Cd, dt=F32)
        O = 2 * Cd
        self.lin_part = e(nd * ((O + 63) // 64) * B * d["ydim"], dt=F32)  # split-K partials of d(embedding)
        eng._build_bwd_tables(self)


class VQVAEEngine:
    def __init__(self, model, device, compute_dtype="fp32"):
        self.m = model
        self.device = torch.device(device)
        self.cd = torch.bfloat16 if compute_dtype in ("bf16", "bfloat16") else F32
        self.dt = ops.dt_code(self.cd)
        L.load()
        enc, dec = model.encoder, model.decoder
        self.dims = d = dict(mel=enc.in_ch, C=enc.ch, Z=enc.z_ch, ns=enc.n_stacks, Cd=dec.ch, S=dec.skip_ch,
                             F=dec.final_ch, cond=dec.cond_ch, nd=dec.n_stacks, K=model.quantizer.z_num,
                             ydim=model.embeds._embedding.weight.shape[1], jitter_p=model.jitter.probability)
        assert d["Z"] == 128 and model.quantizer.z_dim == 128, "the fused VQ kernel is built for z_dim = 128"
        # straight-through VectorQuantizer (use_ema: false)
        self.plain = not model.use_ema
        self.vq_normalize = bool(getattr(model.quantizer, "normalize", False)) if self.plain else False
        self._flatten()
        self._build_layers()
        self._ws = {}
        self.opt_ready = False
        self._enc_gn_separate = os.environ.get("VQX_ENC_GN_FINALIZE") == "1"

    # ------------------------------------------------------------ parameters
    def _flatten(self):
        params = list(self.m.parameters())
        self.params = params
        total = sum(p.numel() for p in params)
        self.flat_p = torch.empty(total, device=self.device, dtype=F32)
        self.flat_g = torch.zeros(total, device=self.device, dtype=F32)
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
        assert all(id(p) in enc_ids for p in params[: len(enc_ids)]), 'encoder parameters must come first'

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
        import bisect
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
        if self.world <= 1:
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

    def _build_layers(self):
        m, d, dev = self.m, self.dims, self.device
        enc, dec = m.encoder.encode, m.decoder
        ns, nd = d["ns"], d["nd"]

        def mk(mod, name, dtype=None):
            kind = 1 if mod.transposed else 0
            Lr = ConvLayer(mod, name, kind, mod.cin, mod.cout, mod.k, mod.k - 1 - mod.padding if kind else mod.padding)
            Lr.wp = torch.empty(Lr.cout, Lr.k * Lr.cin, device=dev, dtype=dtype or self.cd)
            Lr.norm = torch.empty(Lr.rows, device=dev, dtype=F32)
            return Lr

        self.enc0 = mk(enc[0], "encoder.encode.0")
        self.enc_k3 = [mk(enc[i].stack[1], f"encoder.encode.{i}.stack.1") for i in range(1, ns + 1)]
        self.enc_gn = [enc[i].stack[2] for i in range(1, ns + 1)]
        self.enc_sk = [mk(enc[i].skip_layer, f"encoder.encode.{i}.skip_layer") for i in range(1, ns + 1)]
        self.enc_out = mk(enc[ns + 2], f"encoder.encode.{ns + 2}")
        self.dec0 = mk(dec.layers[0], "decoder.layers.0")
        self.dec_in = [mk(dec.layers[i].conv_in, f"decoder.layers.{i}.conv_in") for i in range(1, nd + 1)]
        self.dec_gn = [dec.layers[i].norm_layer for i in range(1, nd + 1)]
        self.dec_cond = [mk(dec.layers[i].conv_cond, f"decoder.layers.{i}.conv_cond", F32) for i in range(1, nd + 1)]
        self.dec_rs = [mk(dec.layers[i].res_skip_layers, f"decoder.layers.{i}.res_skip_layers")
                       for i in range(1, nd + 1)]
        self.fin1 = mk(dec.final_layer[1], "decoder.final_layer.1")
        self.fin2 = mk(dec.final_layer[3], "decoder.final_layer.3")
        self.convs = ([self.enc0] + [x for pair in zip(self.enc_k3, self.enc_sk) for x in pair] + [self.enc_out, self.dec0]
                      + [x for tr in zip(self.dec_in, self.dec_cond, self.dec_rs) for x in tr] + [self.fin1, self.fin2])
        # split-K factors for the wgrad GEMMs: one full round of ~480-512
        # workgroups (2 per CU) at config 2 (64 x 256 frames), at least 4
        # K-tiles (256 frames) per split.  Measured sweep (tools/gemm_bench.py
        # --sweep-splits) on 128 x 128 tiles: dec_in best at 5, enc k3 at 10,
        # res/skip at 24, enc skip at 32 -- exactly floor(512 / tiles).  The
        # tile count comes from the library (3-tap layers use the tap-reuse
        # kernel's 128 x 192 tiles).
        N_ref, T_ref = 64 * 256, 256
        wg_target = int(os.environ.get("VQX_WGRAD_WGS", "512"))  # A/B knobs: workgroups per wgrad launch
        wg_1x1 = int(os.environ.get("VQX_WGRAD_WGS_1X1", str(wg_target)))  # ... for the 1x1 layers
        for Lr in self.convs:
            if Lr in self.dec_cond:
                Lr.splits = 1
                continue
            r, c = (Lr.cin, Lr.cout) if Lr.kind else (Lr.cout, Lr.cin)
            tiles = ops.wgrad_tiles(N_ref, T_ref, r, c, Lr.k, Lr.pad, self.dt)
            Lr.splits = max(1, min((wg_1x1 if Lr.k == 1 else wg_target) // tiles, N_ref // 256))
        # slab arena: one backward group's slabs at a time (kept L2/MALL-resident)
        groups = self._bwd_groups()
        arena = max(sum(Lr.splits * Lr.rows * Lr.cols for Lr in grp) for grp in groups)
        self.arena = torch.empty(arena, device=dev, dtype=F32)
        for grp in groups:
            off = 0
            for Lr in grp:
                n = Lr.splits * Lr.rows * Lr.cols
                Lr.slab = self.arena[off:off + n].view(Lr.splits, Lr.rows, Lr.cols)
                off += n
        self.wn_fwd_table = ops.wn_table([self._wn_entry(Lr, bwd=False) for Lr in self.convs])
        self.groups = groups

    def _bwd_groups(self):
        ns, nd = self.dims["ns"], self.dims["nd"]
        gr = [[self.fin1, self.fin2]]
        gr += [[self.dec_in[i], self.dec_rs[i]] for i in range(nd)]
        gr += [list(self.dec_cond), [self.dec0], [self.enc_out]]
        gr += [[self.enc_k3[i], self.enc_sk[i]] for i in range(ns)]
        gr += [[self.enc0]]
        return gr

    def _wn_entry(self, Lr, bwd):
        mod = Lr.mod
        wn = mod.has_weight_norm
        v = mod.weight_v if wn else mod.weight
        e = dict(v=v, g=mod.weight_g if wn else None, w_packed=Lr.wp, norm=Lr.norm, kind=Lr.kind, cout=Lr.cout,
                 cin=Lr.cin, k=Lr.k, dtype=ops.dt_code(Lr.wp.dtype), splits=Lr.splits)
        if bwd:
            e.update(dv=self.g(v), dg=self.g(mod.weight_g) if wn else None, slabs=Lr.slab)
        return e

    def refresh_tables(self):
        """Rebuild descriptor tables (after remove_weight_norm or a re-flatten)."""
        self.wn_fwd_table = ops.wn_table([self._wn_entry(Lr, bwd=False) for Lr in self.convs])
        for (_, _, train), w in self._ws.items():
            if train:
                self._build_bwd_tables(w)

    def _build_bwd_tables(self, w):
        """Per-workspace backward tables: each group's weight-norm backward plus
        the column reductions of the bias / GroupNorm-affine partials that are
        final when the group's GEMMs are done (one launch per group)."""
        ns, nd, B = self.dims["ns"], self.dims["nd"], w.B
        C, Cd, S = self.dims["C"], self.dims["Cd"], self.dims["S"]
        g = self.g
        cr = ops.colreduce_entry
        cs_enc_b = self._bview(w.colsum_b, B, C)
        dg_enc_b, db_enc_b = self._bview(w.dgam_b, B, C), self._bview(w.dbet_b, B, C)
        dg_dec_b, db_dec_b = self._bview(w.dgam_b, B, 2 * Cd), self._bview(w.dbet_b, B, 2 * Cd)
        t = {}
        f1 = self.fin1
        t["fin"] = [self._wn_entry(f1, True), self._wn_entry(self.fin2, True),
                    cr(w.cs_f1, g(f1.mod.bias))]
        for i in range(nd):
            ci, rs, gn, cond = self.dec_in[i], self.dec_rs[i], self.dec_gn[i], self.dec_cond[i]
            rb = g(rs.mod.bias)
            t[("dec", i)] = [self._wn_entry(ci, True), self._wn_entry(rs, True),
                             cr(w.cs_dec[(nd - 1 - i) % 2], rb[:Cd]), cr(w.cs_skip, rb[Cd:]),
                             cr(w.cs_all[i], g(ci.mod.bias)), cr(dg_dec_b, g(gn.weight)), cr(db_dec_b, g(gn.bias))]
        t["cond"] = [self._wn_entry(Lr, True) for Lr in self.dec_cond]
        t["dec0"] = [self._wn_entry(self.dec0, True), cr(w.cs_dec[nd % 2], g(self.dec0.mod.bias))]
        t["enc_out"] = [self._wn_entry(self.enc_out, True)]
        for i in range(ns):
            k3, sk, gn = self.enc_k3[i], self.enc_sk[i], self.enc_gn[i]
            t[("enc", i)] = [self._wn_entry(k3, True), self._wn_entry(sk, True),
                             cr(w.cs_enc[(ns - 1 - i) % 2], g(sk.mod.bias)),
                             cr(cs_enc_b, g(k3.mod.bias)), cr(dg_enc_b, g(gn.weight)), cr(db_enc_b, g(gn.bias))]
        t["enc0"] = [self._wn_entry(self.enc0, True), cr(w.cs_enc[ns % 2], g(self.enc0.mod.bias))]
        w.bwd_tables = {k: ops.wn_table(v) for k, v in t.items()}
        # parameters whose gradients are final once a group's launch is done
        # (data parallel: their all-reduce is issued right then, parallel/ddp.py)
        w.bwd_params = {k: self._params_written([t_ for e in entries for t_ in (e.get("dv"), e.get("dg"))])
                        for k, entries in t.items()}
        # all ResSkip blocks' conditioning linears, forward and backward, one table
        w.cond_table = ops.linear_table([dict(W=Lr.wp, bias=Lr.mod.bias, out=w.condbias[i], dout=w.cs_all[i],
                                              dW=Lr.slab.view(Lr.rows, Lr.cols), dbias=g(Lr.mod.bias))
                                         for i, Lr in enumerate(self.dec_cond)])

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
        ops.conv_fwd(x, Lr.wp, y, T=T, cin=Lr.cin, cout=Lr.cout, ntaps=Lr.k, pad=Lr.pad, **kw)

    def dgrad(self, Lr, dy, dx, T, **kw):
        ops.conv_dgrad(dy, Lr.wp, dx, T=T, cin=Lr.cout, cout=Lr.cin, ntaps=Lr.k, pad=Lr.pad, **kw)

    def wgrad(self, Lr, dy, x, T, pro=L.PRO_NONE, scale=1.0):
        if Lr.kind == 0:
            ops.conv_wgrad(dy, x, Lr.slab, T=T, r_dim=Lr.cout, c_dim=Lr.cin, ntaps=Lr.k, pad=Lr.pad, shift_sign=1,
                           q_prologue=pro, pro_scale=scale, splits=Lr.splits)
        else:
            assert pro == L.PRO_NONE
            ops.conv_wgrad(x, dy, Lr.slab, T=T, r_dim=Lr.cin, c_dim=Lr.cout, ntaps=Lr.k, pad=Lr.pad, shift_sign=-1,
                           splits=Lr.splits)

    def bias_grad(self, Lr, dy, w):
        ops.colsum(dy, w.cs_part, self.g(Lr.mod.bias))

    # ------------------------------------------------------------ forward
    def pack_weights(self):
        ops.weight_norm_fwd(self.wn_fwd_table)

    def embed_and_cond(self, w, y):
        ops.embedding_fwd(self.m.embeds._embedding.weight, y.reshape(-1), w.yemb)
        if getattr(w, "cond_table", None) is not None:
            Lr = self.dec_cond[0]
            ops.linear_batched_fwd(w.cond_table, w.yemb, w.B, Lr.cin, Lr.cout)
        else:
            for i, Lr in enumerate(self.dec_cond):
                ops.linear_f32(w.yemb, Lr.wp, Lr.mod.bias, w.condbias[i])

    def encoder_fwd(self, w, x_nct):
        T = w.T
        ops.nct_to_ntc(x_nct, w.x)
        # every GEMM producing c_i also writes a_i = LeakyReLU(c_i), the operand
        # of the next k3 conv / the output conv (vqvae.py:86-87 stack[0], 190)
        self.fwd(self.enc0, w.x, w.c[0], T, bias=self.enc0.mod.bias, act=L.PRO_LRELU, y2=w.a[0])
        for i in range(self.dims["ns"]):
            k3, sk, gn = self.enc_k3[i], self.enc_sk[i], self.enc_gn[i]
            if w.fuse_gn:  # statistics of h_i from the k3 GEMM's epilogue tiles, merged inside the skip GEMM
                self.fwd(k3, w.a[i], w.h[i], T, bias=k3.mod.bias, gn_stats=w.gst, gn_groups=1)
                if self._enc_gn_separate:  # A/B: the separate finalize launch
                    ops.gn_finalize_tiles(w.gst, w.N, T, k3.cout, 1, w.enc_mr[i])
                    gkw = {}
                else:
                    gkw = dict(gn_tiles=w.gst)
            else:
                self.fwd(k3, w.a[i], w.h[i], T, bias=k3.mod.bias)
                ops.groupnorm_stats(w.h[i], T, 1, w.gn_part, w.enc_mr[i])
                gkw = {}
            self.fwd(sk, w.c[i], w.c[i + 1], T, bias=sk.mod.bias, gn_h=w.h[i], gn_mr=w.enc_mr[i],
                     gn_gamma=gn.weight, gn_beta=gn.bias, act=L.PRO_LRELU, y2=w.a[i + 1], **gkw)
        self.fwd(self.enc_out, w.a[-1], w.z, T, bias=self.enc_out.mod.bias, out_f32=True)

    def decoder_fwd(self, w, zq_c):
        T, nd, Cd = w.T, self.dims["nd"], self.dims["Cd"]
        self.fwd(self.dec0, zq_c, w.xs[0], T, bias=self.dec0.mod.bias)
        for i in range(nd):
            ci, gn, rs = self.dec_in[i], self.dec_gn[i], self.dec_rs[i]
            if w.fuse_gn:  # statistics from the GEMM's epilogue tiles, finalised inside the GLU launch
                self.fwd(ci, w.xs[i], w.u[i], T, bias=ci.mod.bias, rowbias=w.condbias[i], gn_stats=w.gst, gn_groups=2)
                ops.gn_glu_fwd_tiles(w.u[i], w.g[i], T, w.gst, w.dec_mr[i], gn.weight, gn.bias)
            else:
                self.fwd(ci, w.xs[i], w.u[i], T, bias=ci.mod.bias, rowbias=w.condbias[i])
                ops.groupnorm_stats(w.u[i], T, 2, w.gn_part, w.dec_mr[i])
                ops.gn_glu_fwd(w.u[i], w.g[i], T, w.dec_mr[i], gn.weight, gn.bias)
            self.fwd(rs, w.g[i], w.xs[i + 1], T, bias=rs.mod.bias, res=w.xs[i], out2=w.skip32, split_col=Cd,
                     out2_accumulate=(i > 0))
        # final_layer = ReLU, conv, ReLU, conv on sqrt(1/(nd+1)) * sum(skips) (vqvae.py:316-318)
        ops.scale_act_2d(w.skip32, w.a_skip, math.sqrt(1.0 / (nd + 1)), L.PRO_RELU)
        self.fwd(self.fin1, w.a_skip, w.f1, T, bias=self.fin1.mod.bias, act=L.PRO_RELU)
        self.fwd(self.fin2, w.f1, w.xhat, T, bias=self.fin2.mod.bias, out_f32=True)

    # ------------------------------------------------------------ quantizer host logic
    def _perm_rows(self, n, K, rank_offset=0, n_local=None):
        """torch.randperm(n)[:K] on the CPU generator (layers_vq.py:197,213),
        mapped to local row ids (-1 = row owned by another rank)."""
        perm = torch.randperm(n)[:K]
        if n_local is not None:
            from ..parallel.ddp import owned_rows
            perm = owned_rows(perm, rank_offset, n_local)
        return perm.pin_memory().to(self.device, non_blocking=True)

    def _tile_rows(self, w):
        """N < K path of _tile (layers_vq.py:183-190): repeat z with N(0, 0.01/sqrt(D))
        noise drawn on the CPU generator, then take perm rows.  Host side; rare.
        Data parallel: the tiling runs on the gathered GLOBAL batch (rank
        order = the single-process batch order), and every rank draws the same
        noise and permutation from its identically seeded CPU generator, so all
        ranks hold the single-process global-batch rows."""
        z = w.z.detach()
        if self.world > 1:
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
    def _wn_bwd(self, w, key):
        """A backward group's weight-norm backward + bias/affine reductions;
        its gradients are final afterwards (data parallel: reduce them now)."""
        ops.weight_norm_bwd(w.bwd_tables[key])
        self._grads_final(w.bwd_params[key])

    def _gnb(self, w, i):
        """GNBWD epilogue arguments: the GEMM producing dL/d(GN_i output) also
        writes block i's GroupNorm-backward sums (encoder, G=1)."""
        if not w.fuse_gn:
            return {}
        gn = self.enc_gn[i]
        return dict(gn_bwd=w.gnb_part, gn_h=w.h[i], gn_mr=w.enc_mr[i], gn_gamma=gn.weight, gn_beta=gn.bias,
                    gn_groups=1)

    def _gnb_parts(self, w, cols):
        """GNBWD tiles per utterance (0 = vqx_gn_bwd reduces itself)."""
        return (w.T // 128) * ((cols + 127) // 128) if w.fuse_gn else 0

    def _bview(self, buf, B, C):
        return buf.view(-1)[: B * C].view(B, C)

    def encoder_bwd(self, w, grad_scale=1.0):
        """Backward of beta*z_enc_loss through the encoder: the commitment term is
        the encoder's only gradient source (z_vq is a no-grad gather under
        reduction='frame_mean', layers_vq.py:292,315)."""
        T, N, ns, C = w.T, w.N, self.dims["ns"], self.dims["C"]
        B = w.B
        if not self.plain:  # EMA: the commitment term is the encoder's only gradient
            ops.vq_commit_bwd(w.z, w.zq, 2.0 * self.m.beta * grad_scale / N, w.dz)
        eo = self.enc_out
        self.bias_grad(eo, w.dz, w)
        self.wgrad(eo, w.dz, w.a[ns], T)
        cur = w.dc[0]
        # every dL/dc_i producer also writes its bias-gradient partials (COLSUM)
        # and, for the block below, the GroupNorm-backward sums (GNBWD)
        self.dgrad(eo, w.dz, cur, T, mask=w.a[ns], mask_slope=0.2, colsum=w.cs_enc[0], **self._gnb(w, ns - 1))
        self._wn_bwd(w, "enc_out")
        cs_b, dg_b, db_b = (self._bview(t, B, C) for t in (w.colsum_b, w.dgam_b, w.dbet_b))
        for i in reversed(range(ns)):
            k3, sk, gn = self.enc_k3[i], self.enc_sk[i], self.enc_gn[i]
            j = (ns - i) % 2
            nxt = w.dc[j]
            # cur = dL/dc_{i+1}, the gradient w.r.t. block i's output GN(h_i) + skip(c_i)
            self.wgrad(sk, cur, w.c[i], T)
            ops.gn_bwd(cur, w.h[i], w.dh, T, 1, False, w.enc_mr[i], gn.weight, gn.bias, w.gnb_part, cs_b, dg_b, db_b,
                       nparts=self._gnb_parts(w, C))
            self.wgrad(k3, w.dh, w.a[i], T)
            self.dgrad(k3, w.dh, w.tmp, T, mask=w.a[i], mask_slope=0.2)
            self.dgrad(sk, cur, nxt, T, res=w.tmp, colsum=w.cs_enc[j], **(self._gnb(w, i - 1) if i > 0 else {}))
            # weight norms of k3/sk + biases of sk (cur partials), k3 and the GN affine
            self._wn_bwd(w, ("enc", i))
            cur = nxt
        # cur = dL/dc_0 (conv0 output); conv0's input (the mel batch) needs no gradient
        self.wgrad(self.enc0, cur, w.x, T)
        self._wn_bwd(w, "enc0")

    def decoder_bwd(self, w):
        T, nd, Cd, B = w.T, self.dims["nd"], self.dims["Cd"], w.B
        f1, f2 = self.fin1, self.fin2
        dxhat = w.dxhat
        self.bias_grad(f2, dxhat, w)
        self.wgrad(f2, dxhat, w.f1, T)
        self.dgrad(f2, dxhat, w.df1, T, mask=w.f1, mask_slope=0.0, colsum=w.cs_f1)
        s = math.sqrt(1.0 / (nd + 1))
        self.wgrad(f1, w.df1, w.a_skip, T)
        cur, nxt = w.dr[0], w.dr[1]
        # dL/dskip (identical for every block) -> tail columns of both [dx | dskip] buffers
        self.dgrad(f1, w.df1, cur[:, Cd:], T, mask=w.a_skip, mask_slope=0.0, mask_scale=s, colsum=w.cs_skip)
        ops.convert_2d(cur[:, Cd:], nxt[:, Cd:])
        ops.convert_2d(None, cur, cols=Cd)  # dL/dx_{nd+1} = 0: the last residual output is unused
        ops.zero_(w.cs_dec[0])  # ... and so are its bias-gradient partials (read by block nd-1)
        self._wn_bwd(w, "fin")
        C2 = 2 * Cd
        dg_b, db_b = (self._bview(t, B, C2) for t in (w.dgam_b, w.dbet_b))
        for i in reversed(range(nd)):
            ci, gn, rs = self.dec_in[i], self.dec_gn[i], self.dec_rs[i]
            j = (nd - 1 - i) % 2
            # cur = [dL/dx_{i+1} | dL/dskip]
            self.wgrad(rs, cur, w.g[i], T)
            if w.fuse_gn:  # GLU + GroupNorm backward sums from the res/skip dgrad's epilogue
                self.dgrad(rs, cur, w.dg, T, gn_bwd=w.gnb_part, gn_h=w.u[i], gn_mr=w.dec_mr[i], gn_gamma=gn.weight,
                           gn_beta=gn.bias, gn_groups=2, gn_glu=True)
            else:
                self.dgrad(rs, cur, w.dg, T)
            ops.gn_bwd(w.dg, w.u[i], w.du, T, 2, True, w.dec_mr[i], gn.weight, gn.bias, w.gnb_part, w.cs_all[i],
                       dg_b, db_b, nparts=self._gnb_parts(w, Cd))
            self.wgrad(ci, w.du, w.xs[i], T)
            self.dgrad(ci, w.du, nxt[:, :Cd], T, res=cur[:, :Cd], colsum=w.cs_dec[1 - j])
            # weight norms of conv_in/res_skip + biases of res_skip, conv_in and the GN affine
            self._wn_bwd(w, ("dec", i))
            cur, nxt = nxt, cur
        # speaker conditioning of all blocks at once: dW, bias and d(embedding)
        cond = self.dec_cond[0]
        ops.linear_batched_bwd(w.cond_table, w.yemb, B, cond.cin, cond.cout, w.dyemb, w.lin_part)
        self._wn_bwd(w, "cond")
        dx1 = cur[:, :Cd]  # dL/dx_1, the ConvT0 output
        self.wgrad(self.dec0, dx1, w.zq_in, T)
        if self.plain:  # straight-through VQ: the decoder input's gradient reaches the encoder
            self.dgrad(self.dec0, dx1, w.dzq, T)
        self._wn_bwd(w, "dec0")
        emb_g = self.g(self.m.embeds._embedding.weight)
        ops.zero_(emb_g)
        ops.embedding_bwd(w.dyemb, w.y_dev, emb_g)

    # ------------------------------------------------------------ quantizer
    def vq_init_if_needed(self, w):
        """init_emb (layers_vq.py:192-201) on the first training forward."""
        q = self.m.quantizer
        if q.initialized:
            return False
        K = self.dims["K"]
        if w.N * self.world < K:  # N_global < K: noisy tiling of the global batch (identical on every rank)
            rows = self._tile_rows(w)
            q.embeddings.copy_(rows)
        else:
            perm = self._perm_rows(w.N * self.world, K, self.rank * w.N, w.N if self.world > 1 else None)
            ops.gather_rows(w.z, perm, q.embeddings)
            if self.world > 1:
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
        ops.vq_perplexity(w.bcnt, w.N, w.stats[4:5])

    def vq_plain_backward(self, w):
        """Straight-through + codebook + commitment (+ normalisation) gradients."""
        q = self.m.quantizer
        zin = w.z_norm if self.vq_normalize else w.z
        emb = w.embn if self.vq_normalize else q.embeddings.data
        ops.vq_plain_bwd(w.z, zin, w.z_len if self.vq_normalize else None, w.zq, w.dzq,
                         w.src_t if w.jittered else None, w.T, self.vq_normalize, float(self.m.beta), 2.0 / w.N,
                         w.dz, w.bsum, w.bcnt, emb, w.e_len if self.vq_normalize else None, self.g(q.embeddings))

    def vq_forward_train(self, w):
        if self.plain:
            return self.vq_plain_forward(w)
        q = self.m.quantizer
        K = self.dims["K"]
        self.vq_init_if_needed(w)
        ops.zero_(w.ema)
        ops.vq_forward(w.z, q.embeddings, w.idx, w.zq, w.zq_c, w.stats[1:2], w.vq_part, w.bsum, w.bcnt)
        # rows for dead-code replacement: z[randperm(N)[:K]] (update_emb, layers_vq.py:212-213)
        if w.N * self.world < K:
            rows = self._tile_rows(w)
            if self.rank != 0:  # every rank holds the same rows; the EMA bundle is SUM-reduced
                rows.zero_()
            w.rand_rows.copy_(rows)
        else:
            perm = self._perm_rows(w.N * self.world, K, self.rank * w.N, w.N if self.world > 1 else None)
            ops.gather_rows(w.z, perm, w.rand_rows)
        if self.world > 1:
            self._ema_work = self.comm.all_reduce_sum(w.ema, async_op=True)

    def vq_ema_update(self, w):
        if self.plain:  # the straight-through codebook is a parameter updated by Adam
            return
        q = self.m.quantizer
        if getattr(self, "_ema_work", None) is not None:
            self._ema_work.wait()
            self._ema_work = None
        ops.vq_ema_update(q.emb_sum, q.emb_elem, q.embeddings, w.bsum, w.bcnt, w.rand_rows, q.mu, q.threshold,
                          w.stats[4:8], w.ema_part)

    # ------------------------------------------------------------ full step
    world, rank, comm = 1, 0, None

    def forward_train(self, x, y):
        """Training forward (saves every activation the backward needs).
        x (B, mel, T) f32 device, y (B, 1) int64 device."""
        B, _, T = x.shape
        w = self.ws(B, T, train=True)
        w.y_dev = y.reshape(-1)
        w.x_nct = x
        self.pack_weights()
        self.embed_and_cond(w, w.y_dev)
        self.encoder_fwd(w, x)
        self.vq_forward_train(w)
        w.zq_in = w.zq_c
        w.jittered = False
        if self.dims["jitter_p"] > 0 and self.m.jitter.training:
            src = torch.from_numpy(self.jitter_map(T)).pin_memory()
            w.src_t.copy_(src, non_blocking=True)
            ops.time_gather(w.zq_c, w.zq_j, B, T, w.src_t)
            w.zq_in = w.zq_j
            w.jittered = True
        self.decoder_fwd(w, w.zq_in)
        ops.logloss_fwd_bwd(x, w.xhat, 1.0 / (B * T), w.dxhat, w.stats[0:1], w.loss_part)
        return w

    def backward(self, w, grad_loss=None):
        """Data parallel: every backward group's gradients are all-reduced as
        soon as its weight-norm backward has finalised them (_wn_bwd), so the
        reduces overlap the rest of the backward; the remainder (conditioning,
        ConvT0, embedding, codebook) is flushed at the end."""
        if self.world > 1:
            self._grads_reset()
        if self.plain:
            # straight-through: the encoder's gradient comes through the decoder
            self.decoder_bwd(w)
            self.vq_plain_backward(w)
            self.encoder_bwd(w)
        else:
            self.encoder_bwd(w)
            self.decoder_bwd(w)
        if self.world > 1:
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
        self.exp_avg = torch.zeros(self.n_params, device=dev, dtype=F32)
        self.exp_avg_sq = torch.zeros(self.n_params, device=dev, dtype=F32)
        self.opt_step = torch.zeros(1, device=dev, dtype=torch.int64)
        self.hyper = torch.zeros(16, device=dev, dtype=F32)
        self.sumsq = torch.zeros(1, device=dev, dtype=F32)
        self.norm_part = torch.zeros(1024, device=dev, dtype=F32)
        self.lr0, self.betas, self.eps, self.max_grad_norm = lr, betas, eps, max_grad_norm
        self.sched_step = sched_step or (1 << 30)
        self.sched_gamma = sched_gamma
        self.opt_ready = True

    def optimizer_step(self):
        if self.max_grad_norm > 0:
            ops.grad_sq_norm(self.flat_g, self.norm_part, self.sumsq)
        sumsq = self.sumsq if self.max_grad_norm > 0 else None
        if self.opt_kind == "radam":
            ops.radam_hyper(self.opt_step, self.lr0, self.sched_gamma, self.sched_step, self.betas[0], self.betas[1],
                            self.eps, self.hyper)
            ops.radam_step(self.flat_p, self.flat_g, self.exp_avg, self.exp_avg_sq, self.hyper, sumsq,
                           float(self.max_grad_norm))
            return
        ops.adam_hyper(self.opt_step, self.lr0, self.sched_gamma, self.sched_step, self.betas[0], self.betas[1],
                       self.eps, self.hyper)
        ops.adam_step(self.flat_p, self.flat_g, self.exp_avg, self.exp_avg_sq, self.hyper, sumsq,
                      float(self.max_grad_norm))

    def train_step(self, x, y):
        """One full training step (trainer/basic.py:55-79): forward, backward,
        clip, Adam, StepLR, EMA codebook update.  Returns the device stats
        vector [x_loss, sqerr, -, -, entropy, used_curr, usage, diff_emb]."""
        assert self.opt_ready, "init_optimizer() first"
        w = self.forward_train(x, y)
        self.backward(w)
        self.optimizer_step()
        self.vq_ema_update(w)
        return w

    def total_loss(self, w):
        """(total, VQ loss) device scalars of the step's loss (vqvae.py:83)."""
        n = w.N
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
        n = w.N
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
    def forward_eval(self, x, y):
        """model.eval() forward: no EMA init/update, no jitter (layers_vq.py:282,295,354)."""
        B, _, T = x.shape
        w = self.ws(B, T, train=False) if (B, T, True) not in self._ws else self._ws[(B, T, True)]
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
        """Model.encode (vqvae.py:45-52): encoder + nearest-code index, (B, T) int64."""
        B, _, T = x.shape
        w = self.ws(B, T, train=False) if (B, T, True) not in self._ws else self._ws[(B, T, True)]
        self.pack_weights()
        self.encoder_fwd(w, x)
        q = self.m.quantizer
        if self.plain:
            return q.encode(w.z.view(B, T, -1), time_last=False)
        ops.vq_forward(w.z, q.embeddings, w.idx, None, None, None, w.vq_part, None, None)
        return w.idx.view(B, T).clone()

    def decode(self, z_idx, y):
        """Model.decode (vqvae.py:55-60): codebook gather + decoder, (B, F, T) f32."""
        B, T = z_idx.shape
        w = self.ws(B, T, train=False) if (B, T, True) not in self._ws else self._ws[(B, T, True)]
        w.y_dev = y.reshape(-1)
        self.pack_weights()
        self.embed_and_cond(w, w.y_dev)
        q = self.m.quantizer
        ops.gather_rows(q._codebook() if self.plain else q.embeddings, z_idx.reshape(-1).contiguous(), w.zq)
        ops.convert_2d(w.zq, w.zq_c)
        self.decoder_fwd(w, w.zq_c)
        ops.ntc_to_nct(w.xhat, w.xhat_nct)
        return w.xhat_nct.clone()
