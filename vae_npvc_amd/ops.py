"""Thin tensor-level wrappers over the libvqx C ABI (device tensors in, no
allocation inside the kernels).  Every function here launches HIP kernels on
torch's current stream; there is no CPU path.

Layout convention: activations are frame-major 2-D tensors [N = B*T, C]
(the reference's (B, C, T) transposed), weights of a conv are "packed
effective" [cout, ntaps*cin] (see include/vqx.h).
"""
import ctypes

import torch

from . import _lib as L
from ._lib import call, ptr, stream_ptr

_DT = {torch.float32: L.VQX_F32, torch.bfloat16: L.VQX_BF16}


def dt_code(dtype: torch.dtype) -> int:
    try:
        return _DT[dtype]
    except KeyError:
        raise L.VqxError(f"unsupported dtype {dtype}") from None


def _check_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise L.VqxError("libvqx ops need device tensors (the HIP kernels are the only implementation)")


# ---- host extent checks (debug mode; vae_npvc_amd/debug.py)
_debug = False
_logical_end = {}  # guarded allocations: storage data_ptr -> bytes of the storage that belong to the buffer


def set_debug_checks(on):
    """Check every pointer argument's span against its tensor's storage before
    the calls below (off by default: a few microseconds of host time per call).
    Returns the previous setting."""
    global _debug
    prev, _debug = _debug, bool(on)
    return prev


def _span(t, elems, what):
    """`t` must hold `elems` elements from its data pointer on."""
    if not _debug or t is None or elems <= 0:
        return
    st = t.untyped_storage()
    end = _logical_end.get(st.data_ptr(), st.nbytes())
    avail = (end - t.storage_offset() * t.element_size()) // t.element_size()
    if elems > avail:
        raise L.VqxError(f"extent check: {what} needs {elems} elements from its pointer, its buffer holds {avail}")


def _rows(t, rows, ld, cols, what):
    if rows > 0 and t is not None:
        _span(t, (rows - 1) * ld + cols, what)


def _conv_extents(x, w, y, a, bias, rowbias, res, mask, out2, y2, colsum, stats, tiles, gn_h, gn_mr):
    n, cout, cin = a.n_rows, a.cout, a.cin
    split = a.split_col if out2 is not None else 0
    tm = (n + 127) // 128
    _rows(x, n, a.ldx, cin, "conv x")
    _span(w, cout * a.ntaps * cin, "conv w")
    _rows(y, n, a.ldy, split or cout, "conv y")
    _span(bias, cout, "conv bias")
    _span(rowbias, (n // max(1, a.T)) * cout, "conv rowbias")
    _rows(res, n, a.ldres, split or cout, "conv res")
    _rows(mask, n, a.ldmask, cout, "conv mask")
    _rows(out2, n, a.ldo2, cout - split, "conv out2")
    _rows(y2, n, a.ldy2, cout, "conv y2")
    _span(colsum, tm * cout, "conv colsum_part")
    _span(stats, (n // 128) * ((cout + 127) // 128) * 4, "conv stat_part")
    _span(tiles, (n // 128) * ((cout + 127) // 128) * 4, "conv gn_stat_tiles")
    _rows(gn_h, n, a.ldgn, cout * (2 if a.gn_glu else 1), "conv gn_h")
    _span(gn_mr, (n // max(1, a.T)) * 2 * max(1, a.gn_groups), "conv gn_mean_rstd")


POLICY_AUTO, POLICY_IM2COL, POLICY_TALL256, POLICY_TALL512, POLICY_TR128, POLICY_K1_2PCU = 0, 1, 2, 3, 4, 5  # vqx.h
_policy = POLICY_AUTO


def set_kernel_policy(policy):
    """Policy for the conv GEMM calls that pass no `policy` (include/vqx.h
    VQX_POLICY_*; for tests and A/B tools -- the library itself keeps no such
    state: the policy travels in every call's arguments).  Returns the old one."""
    global _policy
    if policy not in (POLICY_AUTO, POLICY_IM2COL, POLICY_TALL256, POLICY_TALL512, POLICY_TR128, POLICY_K1_2PCU):
        raise ValueError(f"kernel policy {policy} not in 0..5")
    prev, _policy = _policy, int(policy)
    return prev


class kernel_policy:
    """with ops.kernel_policy(p): set_kernel_policy(p) for the block."""

    def __init__(self, policy):
        self.policy = policy

    def __enter__(self):
        self.prev = set_kernel_policy(self.policy)
        return self

    def __exit__(self, *exc):
        set_kernel_policy(self.prev)
        return False


def conv_args(x, w, y, *, T, cin, cout, ntaps, pad, prologue=L.PRO_NONE, pro_scale=1.0, bias=None,
              rowbias=None, res=None, mask=None, mask_slope=0.0, mask_scale=1.0, gn_h=None, gn_mr=None,
              gn_gamma=None, gn_beta=None, out2=None, split_col=0, out2_accumulate=False, out_f32=False,
              act=None, y2=None, colsum=None, gn_stats=None, gn_bwd=None, gn_groups=1, gn_glu=False,
              gn_tiles=None, gn_eps=1e-5, dil=1, policy=None):
    epi = 0
    if bias is not None:
        epi |= L.EPI_BIAS
    if rowbias is not None:
        epi |= L.EPI_ROWBIAS
    if mask is not None:
        epi |= L.EPI_MASK
    if res is not None:
        epi |= L.EPI_RES
    if gn_h is not None and gn_bwd is None:  # GNBWD reads gn_* as the forward GN's operands
        epi |= L.EPI_GNADD
    if out2 is not None:
        epi |= L.EPI_SPLIT
    if out_f32:
        epi |= L.EPI_OUTF32
    if act is not None and y2 is None:
        epi |= L.EPI_ACT
    if y2 is not None:
        epi |= L.EPI_ACT2
    if colsum is not None:
        epi |= L.EPI_COLSUM
    if gn_stats is not None:
        epi |= L.EPI_GNSTATS
    if gn_bwd is not None:
        epi |= L.EPI_GNBWD
    a = L.ConvArgs()
    a.x, a.w, a.y = ptr(x), ptr(w), ptr(y)
    a.bias, a.rowbias, a.res, a.mask = ptr(bias), ptr(rowbias), ptr(res), ptr(mask)
    a.gn_h, a.gn_mean_rstd, a.gn_gamma, a.gn_beta, a.out2 = ptr(gn_h), ptr(gn_mr), ptr(gn_gamma), ptr(gn_beta), ptr(out2)
    a.n_rows, a.T, a.cin, a.cout, a.ntaps, a.pad, a.dil = x.shape[0], T, cin, cout, ntaps, pad, dil
    a.kernel_policy = _policy if policy is None else policy
    a.ldx, a.ldy = x.stride(0), y.stride(0)
    a.ldres = res.stride(0) if res is not None else 0
    a.ldmask = mask.stride(0) if mask is not None else 0
    a.ldgn = gn_h.stride(0) if gn_h is not None else 0
    a.ldo2 = out2.stride(0) if out2 is not None else 0
    a.dtype = dt_code(x.dtype)
    a.prologue, a.epilogue = prologue, epi
    a.split_col, a.out2_accumulate = split_col, int(bool(out2_accumulate))
    a.pro_scale, a.mask_slope, a.mask_scale = pro_scale, mask_slope, mask_scale
    a.y2, a.ldy2 = ptr(y2), (y2.stride(0) if y2 is not None else 0)
    a.epi_act = act if act is not None else 0
    a.colsum_part = ptr(colsum)
    a.gn_stat_tiles, a.gn_eps = ptr(gn_tiles), gn_eps
    a.stat_part = ptr(gn_stats if gn_stats is not None else gn_bwd)
    a.gn_groups, a.gn_glu = gn_groups, int(gn_glu)
    if _debug:
        _conv_extents(x, w, y, a, bias, rowbias, res, mask, out2, y2, colsum,
                      gn_stats if gn_stats is not None else gn_bwd, gn_tiles, gn_h, gn_mr)
    return a


class LaunchProbe:
    """Per-launch timing of the conv GEMM kernels (bench.py's roofline leg).
    libvqx launches each GEMM with hipExtLaunchKernelGGL and a start/stop
    event pair stamped on the kernel's own dispatch (vqx_probe_*), on the
    stream the kernel runs on; this class only labels and aggregates."""

    _DT = {L.VQX_F32: "float", L.VQX_BF16: "unsigned short"}

    def __init__(self):
        self.shapes = []

    def clear(self):
        self.shapes = []
        call("vqx_probe_clear")

    def start(self):
        """Resume recording (the log is kept; clear() empties it)."""
        call("vqx_probe_enable", 1)

    def stop(self):
        call("vqx_probe_enable", 0)

    def select(self, info=None):
        """Record only launches of the kernel with this 5-int info (records()[i][4]);
        None = all.  Other launches skip the event pair and its queue cost."""
        if info is None:
            call("vqx_probe_select", None)
        else:
            self._sel = (ctypes.c_int32 * 5)(*info)
            call("vqx_probe_select", self._sel)

    def records(self):
        """[(rocprof symbol, flops, seconds, shape label, info5)] after a device sync."""
        torch.cuda.synchronize()
        n = ctypes.c_int64()
        call("vqx_probe_count", ctypes.byref(n))
        info = (ctypes.c_int32 * 5)()
        fl, ms = ctypes.c_double(), ctypes.c_float()
        out = []
        for i in range(n.value):
            call("vqx_probe_read", i, info, ctypes.byref(fl), ctypes.byref(ms))
            dt, mode, pro, gen, ek = list(info)  # ek: epilogue kind (vqx_gemm_kernel.h EK_*)
            bk = 64 if dt == L.VQX_BF16 else 32
            if gen == 5:  # data + weight gradient in one launch (vqx_gemm_dual.hip)
                sym = {2: f"vqx::dual_tr_kernel<{ek}>", 3: f"vqx::dual_k1_kernel<{ek}>"}.get(pro, "vqx::dual_kernel")
            elif gen == 4:  # three workgroups per CU (vqx_gemm_kernel.h conv_gemm3_kernel)
                sym = f"vqx::conv_gemm3_kernel<{self._DT[dt]}, {mode}, {pro}, false, {ek}>"
            elif gen == 6:  # ping-pong tap-reuse kernel (vqx_gemm_pp.h conv_pp_kernel)
                sym = f"vqx::conv_pp_kernel<{mode}, {ek}, {pro}, 2>"  # pro slot = frame segments
            elif gen == 2 and mode == 2:  # tap-reuse weight gradient (vqx_gemm_kernel.h wgrad_tr_kernel)
                sym = f"vqx::wgrad_tr_kernel<{ek}, {pro}>"  # pro slot = K groups
            elif gen == 3:  # tall tap-reuse kernel (vqx_gemm_kernel.h conv_tr8_kernel)
                sym = f"vqx::conv_tr8_kernel<{mode}, {ek}, {pro}>"  # pro slot = frame segments
            elif gen == 2:  # tap-reuse kernel (3-tap FWD/DGRAD, vqx_gemm_kernel.h conv_tr_kernel)
                sym = f"vqx::conv_tr_kernel<{mode}, {ek}, {pro}>"  # pro slot = channels per stage
            else:
                sym = f"vqx::conv_gemm_kernel<{self._DT[dt]}, {mode}, {pro}, {'true' if gen else 'false'}, {bk}, 2, {ek}>"
            out.append((sym, fl.value, ms.value * 1e-3, self.shapes[i] if i < len(self.shapes) else "",
                        (dt, mode, pro, gen, ek)))
        return out

    def summary(self, by_shape=False):
        """Aggregate per kernel symbol (by_shape: per symbol and layer shape)."""
        agg = {}
        for key, fl, sec, shape, _ in self.records():
            if by_shape:
                key = f"{key} {shape}"
            a = agg.setdefault(key, [0, 0.0, 0.0])
            a[0] += 1
            a[1] += fl
            a[2] += sec
        return {k: {"launches": n, "flops": f, "seconds": t, "avg_us": 1e6 * t / n, "tflops": f / t / 1e12}
                for k, (n, f, t) in agg.items()}


_probe = None


def set_probe(p):
    """Install (p.start()) or remove (None) the GEMM launch probe."""
    global _probe
    if _probe is not None and p is None:
        _probe.stop()
    _probe = p
    if p is not None:
        p.start()


def conv_fwd(x, w, y, **kw):
    """y = epi(conv(pro(x), w)); x [N, cin], w packed [cout, ntaps*cin], y [N, cout]."""
    _check_cuda(x, w, y)
    a = conv_args(x, w, y, **kw)
    if _probe is not None:
        _probe.shapes.append(f"{a.cin}->{a.cout} k{a.ntaps} epi{a.epilogue}")
    call("vqx_conv1d_fwd", ctypes.byref(a), stream_ptr())
    return y


def conv_dgrad(dy, w, dx, **kw):
    """dx = epi(conv_transpose(dy, w)); dy [N, cout_f], w packed [cout_f, ntaps*cin_f], dx [N, cin_f].
    Pass cin=cout_f, cout=cin_f."""
    _check_cuda(dy, w, dx)
    a = conv_args(dy, w, dx, **kw)
    if _probe is not None:
        _probe.shapes.append(f"{a.cin}->{a.cout} k{a.ntaps} epi{a.epilogue}")
    call("vqx_conv1d_dgrad", ctypes.byref(a), stream_ptr())
    return dx


def wgrad_args(p, q, slabs, *, T, r_dim, c_dim, ntaps, pad, shift_sign=1, q_prologue=L.PRO_NONE, pro_scale=1.0,
               splits=1, dil=1, policy=None, fixup_dw=None, fixup_counters=None):
    a = L.WgradArgs()
    a.kernel_policy = _policy if policy is None else policy
    a.p, a.q, a.slabs = ptr(p), ptr(q), ptr(slabs)
    a.n_rows, a.T, a.r_dim, a.c_dim, a.ntaps, a.pad, a.shift_sign = p.shape[0], T, r_dim, c_dim, ntaps, pad, shift_sign
    a.ldp, a.ldq = p.stride(0), q.stride(0)
    a.dtype, a.q_prologue, a.splits, a.pro_scale, a.dil = dt_code(p.dtype), q_prologue, splits, pro_scale, dil
    a.slab_dtype = dt_code(slabs.dtype)
    a.fixup_dw, a.fixup_counters = ptr(fixup_dw), ptr(fixup_counters)
    if _debug:
        _span(fixup_dw, r_dim * ntaps * c_dim, "wgrad fixup_dw")
        _rows(p, a.n_rows, a.ldp, r_dim, "wgrad p")
        _rows(q, a.n_rows, a.ldq, c_dim, "wgrad q")
        _span(slabs, splits * r_dim * ntaps * c_dim, "wgrad slabs")
    return a


def conv_wgrad(p, q, slabs, **kw):
    """slabs[s, r, j*c_dim + c] = sum_{n in split s} p[n, r] * pro(q[n + sign*(j*dil-pad), c]);
    slabs fp32, or bf16 for bf16 operands (each split's partial rounded once).
    Keywords: T, r_dim, c_dim, ntaps, pad, shift_sign, q_prologue, pro_scale, splits, dil."""
    _check_cuda(p, q, slabs)
    a = wgrad_args(p, q, slabs, **kw)
    if _probe is not None:
        _probe.shapes.append(f"{a.r_dim}x{a.ntaps}x{a.c_dim} s{a.splits}")
    call("vqx_conv1d_wgrad", ctypes.byref(a), stream_ptr())
    return slabs


def conv_dgrad_wgrad(dy, w, dx, dgrad_kw, p, q, slabs, wgrad_kw):
    """conv_wgrad(p, q, slabs, **wgrad_kw) and conv_dgrad(dy, w, dx, **dgrad_kw)
    of one layer (same output gradient) through vqx_conv1d_dgrad_wgrad: one
    launch interleaving both GEMMs where a fused kernel covers the pair, else
    the two launches in that order.  Returns True when fused."""
    _check_cuda(dy, w, dx, p, q, slabs)
    ad = conv_args(dy, w, dx, **dgrad_kw)
    aw = wgrad_args(p, q, slabs, **wgrad_kw)
    fused = ctypes.c_int32(0)
    call("vqx_conv1d_dgrad_wgrad", ctypes.byref(ad), ctypes.byref(aw), ctypes.byref(fused), stream_ptr())
    if _probe is not None:
        sd = f"{ad.cin}->{ad.cout} k{ad.ntaps} epi{ad.epilogue}"
        sw = f"{aw.r_dim}x{aw.ntaps}x{aw.c_dim} s{aw.splits}"
        _probe.shapes.extend([f"dual {sd} + {sw}"] if fused.value else [sw, sd])
    return bool(fused.value)


def wgrad_tiles(n_rows, T, r_dim, c_dim, ntaps, pad, dtype, q_prologue=L.PRO_NONE, dil=1, policy=POLICY_AUTO):
    """Output tiles per split of the weight-gradient kernel conv_wgrad would
    launch under kernel policy `policy`."""
    t = ctypes.c_int32()
    call("vqx_wgrad_tiles", n_rows, T, r_dim, c_dim, ntaps, pad, dil, dtype, q_prologue, policy, ctypes.byref(t))
    return t.value


def _wn_extents(d):
    """Spans of one weight-norm table entry (include/vqx.h vqx_wn_layer)."""
    kind, cout, cin, k, s = d["kind"], d["cout"], d["cin"], d["k"], d.get("stride", 1) or 1
    if kind == L.WN_COLREDUCE:
        _span(d.get("v"), cin * cout, "colreduce src")
        _span(d.get("dv"), cout, "colreduce dst")
        return
    rows = cin if kind in (1, L.WN_RESAMPLE_T) else cout
    cols = (3 * s * cin if kind == L.WN_RESAMPLE else 3 * s * cout if kind == L.WN_RESAMPLE_T
            else (cout if kind == 1 else cin) * k)
    for key in ("v", "dv"):
        _span(d.get(key), cout * cin * k, f"weight-norm {key}")
    for key in ("g", "dg", "norm"):
        _span(d.get(key), rows, f"weight-norm {key}")
    _span(d.get("w_packed"), rows * cols, "weight-norm w_packed")
    _span(d.get("slabs"), d.get("splits", 1) * rows * cols, "weight-norm slabs")


def wgrad_fixup_ok(n_rows, T, r_dim, c_dim, ntaps, pad, dtype, slab_dtype, q_prologue=L.PRO_NONE, dil=1,
                   policy=POLICY_AUTO):
    """Whether conv_wgrad of this shape takes the in-launch split-K reduction (fixup_dw, ABI 127)."""
    ok = ctypes.c_int32()
    call("vqx_wgrad_fixup_ok", n_rows, T, r_dim, c_dim, ntaps, pad, dil, dtype, slab_dtype, q_prologue, policy,
         ctypes.byref(ok))
    return bool(ok.value)


def wn_table(layers):
    """Pack a list of dicts into a ctypes WNLayer array (host copy) and a device byte tensor copy."""
    arr = (L.WNLayer * len(layers))()
    for i, d in enumerate(layers):
        e = arr[i]
        for k in ("v", "g", "w_packed", "norm", "dv", "dg", "slabs"):
            setattr(e, k, ptr(d.get(k)))
        e.kind, e.cout, e.cin, e.k = d["kind"], d["cout"], d["cin"], d["k"]
        e.splits, e.dtype = d.get("splits", 1), d["dtype"]
        e.stride, e.pad = d.get("stride", 0), d.get("pad", 0)
        sl = d.get("slabs")
        e.slab_dtype = dt_code(sl.dtype) if sl is not None else L.VQX_F32
        if _debug:
            _wn_extents(d)
    raw = bytes(arr)
    dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to("cuda")
    return arr, dev


def colreduce_entry(src, dst):
    """VQX_WN_COLREDUCE table entry: dst[c] = sum_r src[r][c] (src contiguous f32 [R][C])."""
    R, C = src.shape
    return dict(kind=L.WN_COLREDUCE, v=src, dv=dst, cin=R, cout=C, k=1, dtype=L.VQX_F32, splits=1)


def linear_table(layers):
    """Device table of vqx_linear_layer (host ctypes copy kept alive alongside)."""
    arr = (L.LinearLayer * len(layers))()
    for i, d in enumerate(layers):
        for k in ("W", "bias", "out", "dout", "dW", "dbias"):
            setattr(arr[i], k, ptr(d.get(k)))
    arr.ents = layers  # the tensors behind the pointers (debug extent checks)
    dev = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to("cuda")
    return arr, dev


def _linear_extents(arr, B, I, O, dc=None, partials=None):
    if not _debug:
        return
    for d in arr.ents:
        _span(d.get("W"), O * I, "linear W")
        _span(d.get("dW"), O * I, "linear dW")
        for key in ("bias", "dbias"):
            _span(d.get(key), O, f"linear {key}")
        for key in ("out", "dout"):
            _span(d.get(key), B * O, f"linear {key}")
    _span(dc, B * I, "linear dc")
    _span(partials, len(arr) * ((O + 63) // 64) * B * I, "linear partials")


def linear_batched_fwd(table, c, B, I, O):
    arr, dev = table
    _linear_extents(arr, B, I, O)
    _span(c, B * I, "linear c")
    call("vqx_linear_batched_fwd", dev.data_ptr(), len(arr), ptr(c), B, I, O, stream_ptr())


def linear_ids_ok(B, I, O, emb):
    """Whether linear_batched_*_ids take this shape (vqx.h: I = 128, B <= 64, O % 64 == 0, aligned table)."""
    return I == 128 and 1 <= B <= 64 and O % 64 == 0 and emb.data_ptr() % 16 == 0


def linear_batched_fwd_ids(table, emb, ids, B, I, O):
    """linear_batched_fwd with c[b] = emb[ids[b]] (the embedding lookup in the operand loads)."""
    arr, dev = table
    _check_cuda(emb, ids)
    if ids.dtype != torch.int64 or ids.numel() != B:
        raise ValueError("linear_batched_fwd_ids: B int64 ids")
    _linear_extents(arr, B, I, O)
    call("vqx_linear_batched_fwd_ids", dev.data_ptr(), len(arr), ptr(emb), ptr(ids), B, I, O, stream_ptr())


def linear_batched_bwd_ids(table, emb, ids, B, I, O, dc, partials):
    arr, dev = table
    _check_cuda(emb, ids)
    if ids.dtype != torch.int64 or ids.numel() != B:
        raise ValueError("linear_batched_bwd_ids: B int64 ids")
    _linear_extents(arr, B, I, O, dc, partials)
    call("vqx_linear_batched_bwd_ids", dev.data_ptr(), len(arr), ptr(emb), ptr(ids), B, I, O, ptr(dc), ptr(partials),
         stream_ptr())


def linear_batched_bwd(table, c, B, I, O, dc, partials=None):
    """partials: f32 workspace of >= len(table) * ceil(O/64) * B * I (allocated if None)."""
    arr, dev = table
    if dc is not None and partials is None:
        partials = torch.empty(len(arr) * ((O + 63) // 64) * B * I, device=c.device, dtype=torch.float32)
    _linear_extents(arr, B, I, O, dc, partials)
    _span(c, B * I, "linear c")
    call("vqx_linear_batched_bwd", dev.data_ptr(), len(arr), ptr(c), B, I, O, ptr(dc), ptr(partials), stream_ptr())


WNF_NORMS_READY = 1  # include/vqx.h VQX_WNF_NORMS_READY


def weight_norm_fwd(table, flags=0):
    arr, dev = table
    if flags:
        call("vqx_weight_norm_fwd_flags", ctypes.addressof(arr), dev.data_ptr(), len(arr), flags, stream_ptr())
    else:
        call("vqx_weight_norm_fwd", ctypes.addressof(arr), dev.data_ptr(), len(arr), stream_ptr())


def weight_norm_bwd(table, sq_partials=None):
    """sq_partials: also leave the sum of squares of every written gradient
    value as per-wave partials there (weight_norm_bwd_partials(table) floats)."""
    arr, dev = table
    if sq_partials is None:
        call("vqx_weight_norm_bwd", ctypes.addressof(arr), dev.data_ptr(), len(arr), stream_ptr())
        return
    _check_cuda(sq_partials)
    if _debug:
        _span(sq_partials, weight_norm_bwd_partials(table), "weight-norm sq partials")
    call("vqx_weight_norm_bwd_sq", ctypes.addressof(arr), dev.data_ptr(), len(arr), ptr(sq_partials),
         sq_partials.numel(), stream_ptr())


def weight_norm_bwd_partials(table):
    """Number of sum-of-squares partials weight_norm_bwd(table, sq) writes."""
    arr, _ = table
    n = ctypes.c_int64(0)
    call("vqx_weight_norm_bwd_partials", ctypes.addressof(arr), len(arr), ctypes.byref(n))
    return n.value


def sq_norm_finish(partials, g, ranges, out, scratch):
    """out[0] = sum(partials) + sum over ranges (int64 [n, 2] device tensor of
    (offset, length) into g) of g^2, in a fixed order; scratch >= 256 floats."""
    _check_cuda(partials, g, out, scratch)
    if scratch.numel() < 256:
        raise ValueError("sq_norm_finish: scratch needs 256 floats")
    nr = 0 if ranges is None else ranges.shape[0]
    if nr:
        _check_cuda(ranges)
        if ranges.dtype != torch.int64 or ranges.dim() != 2 or ranges.shape[1] != 2:
            raise ValueError("sq_norm_finish: ranges must be an int64 [n, 2] tensor")
    call("vqx_sq_norm_finish", ptr(partials), partials.numel(), ptr(g), ptr(ranges) if nr else None, nr, ptr(scratch),
         ptr(out), stream_ptr())
    return out


def sq_norm_finish_adam(partials, g, ranges, out, scratch, step, lr0, gamma, step_size, beta1, beta2, eps, hyper):
    """sq_norm_finish then adam_hyper, the second in the finish's last launch."""
    _check_cuda(partials, g, out, scratch, step, hyper)
    if scratch.numel() < 256:
        raise ValueError("sq_norm_finish_adam: scratch needs 256 floats")
    nr = 0 if ranges is None else ranges.shape[0]
    if nr:
        _check_cuda(ranges)
        if ranges.dtype != torch.int64 or ranges.dim() != 2 or ranges.shape[1] != 2:
            raise ValueError("sq_norm_finish_adam: ranges must be an int64 [n, 2] tensor")
    call("vqx_sq_norm_finish_adam", ptr(partials), partials.numel(), ptr(g), ptr(ranges) if nr else None, nr,
         ptr(scratch), ptr(out), ptr(step), lr0, gamma, step_size, beta1, beta2, eps, ptr(hyper), stream_ptr())
    return out


def groupnorm_stats(x, T, G, partials, mean_rstd, eps=1e-5):
    call("vqx_groupnorm_stats", ptr(x), x.stride(0), dt_code(x.dtype), x.shape[0], T, x.shape[1], G, eps,
         ptr(partials), ptr(mean_rstd), stream_ptr())
    return mean_rstd


def gn_lrelu_fwd(h, g, T, mean_rstd, gamma, beta):
    """g = LeakyReLU_0.2(GroupNorm_1(h)) with precomputed statistics mean_rstd [B, 2]."""
    call("vqx_gn_lrelu_fwd", ptr(h), h.stride(0), ptr(g), g.stride(0), dt_code(h.dtype), h.shape[0], T, h.shape[1],
         ptr(mean_rstd), ptr(gamma), ptr(beta), stream_ptr())


def gn_glu_fwd(u, g, T, mean_rstd, gamma, beta):
    call("vqx_gn_glu_fwd", ptr(u), u.stride(0), ptr(g), g.stride(0), dt_code(u.dtype), u.shape[0], T, u.shape[1],
         ptr(mean_rstd), ptr(gamma), ptr(beta), stream_ptr())
    return g


def gn_glu_fwd_tiles(u, g, T, parts, mean_rstd, gamma, beta, eps=1e-5):
    """gn_finalize_tiles(G=2) + gn_glu_fwd in one launch; writes mean_rstd."""
    call("vqx_gn_glu_fwd_tiles", ptr(u), u.stride(0), ptr(g), g.stride(0), dt_code(u.dtype), u.shape[0], T,
         u.shape[1], ptr(parts), eps, ptr(mean_rstd), ptr(gamma), ptr(beta), stream_ptr())
    return g


def gn_bwd(dy, u, du, T, G, glu, mean_rstd, gamma, beta, partials, colsum_b=None, dgamma_b=None, dbeta_b=None,
           nparts=0):
    """nparts > 0: `partials` already holds the producing GEMM's GNBWD tiles (nparts per utterance)."""
    call("vqx_gn_bwd", ptr(dy), dy.stride(0), ptr(u), u.stride(0), ptr(du), du.stride(0), dt_code(u.dtype),
         u.shape[0], T, u.shape[1], G, int(glu), ptr(mean_rstd), ptr(gamma), ptr(beta), ptr(partials), nparts,
         ptr(colsum_b), ptr(dgamma_b), ptr(dbeta_b), stream_ptr())
    return du


def gn_finalize_tiles(parts, n_rows, T, C, G, mean_rstd, eps=1e-5):
    call("vqx_gn_finalize_tiles", ptr(parts), n_rows, T, C, G, eps, ptr(mean_rstd), stream_ptr())
    return mean_rstd


def colsum(x, partials, out, accumulate=False, C=None):
    C = x.shape[1] if C is None else C
    call("vqx_colsum", ptr(x), x.stride(0), dt_code(x.dtype), x.shape[0], C, ptr(partials), ptr(out),
         int(accumulate), stream_ptr())
    return out


def colsum_parts(n_rows, C, dtype):
    """Row parts colsum_partials writes for an [n_rows, C] input of `dtype`."""
    n = ctypes.c_int32()
    call("vqx_colsum_parts", int(n_rows), int(C), dt_code(dtype), ctypes.byref(n))
    return n.value


def colsum_partials(x, partials):
    """partials[p][c] = sum over row part p of x[:, c] (the first level of colsum);
    `partials` is f32 [colsum_parts(...), C], to be reduced later (colreduce_entry)."""
    _check_cuda(x, partials)
    n, C = x.shape
    if tuple(partials.shape) != (colsum_parts(n, C, x.dtype), C) or not partials.is_contiguous():
        raise ValueError(f"colsum_partials: partials {tuple(partials.shape)} != ({colsum_parts(n, C, x.dtype)}, {C})")
    call("vqx_colsum_partials", ptr(x), x.stride(0), dt_code(x.dtype), n, C, ptr(partials), stream_ptr())
    return partials


def nct_to_ntc(x_nct, y):
    B, C, T = x_nct.shape
    call("vqx_nct_to_ntc", ptr(x_nct), B, C, T, ptr(y), y.stride(0), dt_code(y.dtype), stream_ptr())
    return y


def step_prologue(wn_table=None, cond=None, x_nct=None, y=None):
    """One launch for weight_norm_fwd(wn_table, flags=WNF_NORMS_READY),
    linear_batched_fwd_ids(*cond) and nct_to_ntc(x_nct, y), with their bits
    (vqx_step_prologue).  cond = (table, emb, ids, B, I, O); any job may be None."""
    wh, wd, nw = None, 0, 0
    if wn_table is not None:
        arr, dev = wn_table
        wh, wd, nw = ctypes.addressof(arr), dev.data_ptr(), len(arr)
    cd, nc, emb_p, ids_p, B, I, O = 0, 0, 0, 0, 0, 0, 0
    if cond is not None:
        (arr, dev), emb, ids, B, I, O = cond
        _check_cuda(emb, ids)
        if ids.dtype != torch.int64 or ids.numel() != B:
            raise ValueError("step_prologue: B int64 ids")
        _linear_extents(arr, B, I, O)
        cd, nc, emb_p, ids_p = dev.data_ptr(), len(arr), ptr(emb), ptr(ids)
    xp, xB, C, T, yp, ldy, ydt = 0, 0, 0, 0, 0, 0, 0
    if x_nct is not None:
        _check_cuda(x_nct, y)
        xB, C, T = x_nct.shape
        if not x_nct.is_contiguous() or y.dim() != 2 or y.shape[0] != xB * T or y.shape[1] < C or y.stride(1) != 1:
            raise ValueError(f"step_prologue: x {tuple(x_nct.shape)} into y {tuple(y.shape)}")
        xp, yp, ldy, ydt = ptr(x_nct), ptr(y), y.stride(0), dt_code(y.dtype)
    call("vqx_step_prologue", wh, wd, nw, cd, nc, emb_p, ids_p, B, I, O, xp, xB, C, T, yp, ldy, ydt, stream_ptr())


def ntc_to_nct(y, x_nct):
    B, C, T = x_nct.shape
    call("vqx_ntc_to_nct", ptr(y), y.stride(0), dt_code(y.dtype), B, C, T, ptr(x_nct), stream_ptr())
    return x_nct


def logloss_fwd_bwd(x_nct, xhat, grad_scale, dxhat, loss_out, partials):
    B, C, T = x_nct.shape
    call("vqx_logloss_fwd_bwd", ptr(x_nct), ptr(xhat), xhat.stride(0), B, C, T, grad_scale, ptr(dxhat),
         dxhat.stride(0) if dxhat is not None else 0, dt_code(dxhat.dtype) if dxhat is not None else 0,
         ptr(loss_out), ptr(partials), stream_ptr())
    return loss_out


def logloss_parts(x_nct, xhat, grad_scale, dxhat, partials):
    """logloss_fwd_bwd without its final sum launch: the per-workgroup partials
    only; returns their count (vq_ema_update(close=...) sums them)."""
    B, C, T = x_nct.shape
    n = ctypes.c_int32(0)
    call("vqx_logloss_parts", ptr(x_nct), ptr(xhat), xhat.stride(0), B, C, T, grad_scale, ptr(dxhat),
         dxhat.stride(0) if dxhat is not None else 0, dt_code(dxhat.dtype) if dxhat is not None else 0,
         ptr(partials), ctypes.byref(n), stream_ptr())
    if n.value > partials.numel():
        raise L.VqxError(f"logloss_parts: {n.value} partials written into a buffer of {partials.numel()}")
    return n.value


def logloss_fwd_bwd_x(x_nct, xhat, grad_scale, dxhat, loss_out, partials, extra_partials, extra_out):
    """logloss_fwd_bwd, and extra_out[0] = the sum of extra_partials in the same
    final launch (the VQ kernel's commitment partials: VQ_FRAMES frames each)."""
    B, C, T = x_nct.shape
    _check_cuda(extra_partials, extra_out)
    call("vqx_logloss_fwd_bwd_x", ptr(x_nct), ptr(xhat), xhat.stride(0), B, C, T, grad_scale, ptr(dxhat),
         dxhat.stride(0) if dxhat is not None else 0, dt_code(dxhat.dtype) if dxhat is not None else 0,
         ptr(loss_out), ptr(partials), ptr(extra_partials), extra_partials.numel(), ptr(extra_out), stream_ptr())
    return loss_out


VQ_FRAMES = 32  # frames per commitment partial of vqx_vq_forward (vqx_vq.hip VQ_FRAMES)


def vq_workspace(n_rows, K, stats, D=128):
    """Floats of workspace vqx_vq_forward needs for K codes of width D (with or
    without EMA statistics)."""
    out = ctypes.c_int64()
    call("vqx_vq_workspace", int(n_rows), int(K), int(D), int(bool(stats)), ctypes.byref(out))
    return out.value


def vq_forward(z, E, idx, zq, zq_c, sqerr, partials=None, bsum=None, bcnt=None):
    """partials: f32 workspace of >= vq_workspace(N, K, bsum is not None, D) floats (allocated if None)."""
    N, D = z.shape
    need = vq_workspace(N, E.shape[0], bsum is not None, D)
    if partials is None:
        partials = torch.empty(need, device=z.device, dtype=torch.float32)
    if partials.numel() < need:
        raise ValueError(f"vq_forward: workspace {partials.numel()} < {need} floats")
    if _debug:
        K = E.shape[0]
        for t, n, what in ((idx, N, "idx"), (zq, N * D, "zq"), (zq_c, N * D, "zq_c"), (bsum, K * D, "bsum"),
                           (bcnt, K, "bcnt"), (E, K * D, "codebook")):
            _span(t, n, f"vq_forward {what}")
    call("vqx_vq_forward", ptr(z), N, D, ptr(E), E.shape[0], ptr(idx), ptr(zq), ptr(zq_c),
         dt_code(zq_c.dtype) if zq_c is not None else 0, ptr(sqerr), ptr(partials), ptr(bsum), ptr(bcnt),
         stream_ptr())


def vq_stats(z, idx, K, partials, bsum, bcnt):
    """EMA statistics alone (vqx_vq_stats): bsum [K, D] = sum of the frames per
    code, bcnt [K] = counts; partials as vq_forward's workspace with stats."""
    N, D = z.shape
    need = vq_workspace(N, K, True, D)
    if partials.numel() < need:
        raise ValueError(f"vq_stats: workspace {partials.numel()} < {need} floats")
    call("vqx_vq_stats", ptr(z), N, D, ptr(idx), K, ptr(partials), ptr(bsum), ptr(bcnt), stream_ptr())


def ema_workspace(K, D):
    """Floats of vq_ema_update's workspace: the per-workgroup partials and the arrival counter."""
    return (K * D + 1023) // 1024 + 1


def vq_ema_update(emb_sum, emb_elem, E, bsum, bcnt, rand_rows, mu, threshold, diag, partials=None, clear=False,
                  sums=(), publish=None, rows=None):
    """partials: workspace of ceil(K*D/1024) + 1 floats, zero-initialised once
    (the last word is an arrival counter each call leaves zero; allocated here
    if None); clear: bsum / bcnt are zero afterwards (vqx_vq_ema_update_clear).
    sums: up to two (parts, scale, out) -- out[0] = scale * sum(parts) in the
    last workgroup; publish: (mailbox, src, dev_copy) -- src published into the
    Mailbox after them; rows: (src, host int32 indices) -- rand_rows read as
    src[indices] inside the launch (rand_rows unused) (vqx_vq_ema_update_close,
    which implies clear).  Returns publish's (seq, slot), else None."""
    K, D = E.shape
    need = ema_workspace(K, D)
    if partials is None:
        partials = torch.zeros(need, device=E.device, dtype=torch.float32)
    if partials.numel() < need:
        raise ValueError(f"vq_ema_update: workspace {partials.numel()} < {need} floats")
    if _debug:
        for t, n, what in ((emb_sum, K * D, "emb_sum"), (emb_elem, K, "emb_elem"), (bsum, K * D, "bsum"),
                           (bcnt, K, "bcnt"), (rand_rows, K * D, "rand_rows"), (diag, 4, "diag")):
            _span(t, n, f"vq_ema_update {what}")
    if not sums and publish is None and rows is None:
        call("vqx_vq_ema_update_clear" if clear else "vqx_vq_ema_update", ptr(emb_sum), ptr(emb_elem), ptr(E), ptr(bsum),
             ptr(bcnt), ptr(rand_rows), K, D, mu, threshold, ptr(diag), ptr(partials), stream_ptr())
        return None
    if not clear or len(sums) > 2:
        raise ValueError("vq_ema_update: sums / publish need clear=True and at most two sums")
    c = L.StepClose()
    for i, (parts, scale, out) in enumerate(sums):
        _check_cuda(parts, out)
        c.parts[i], c.n[i], c.scale[i], c.out[i] = ptr(parts), parts.numel(), float(scale), ptr(out)
    res = None
    if publish is not None:
        mb, src, copy = publish
        _check_cuda(src, copy)
        if src.numel() > mb.floats or not src.is_contiguous() or src.dtype != torch.float32:
            raise ValueError(f"vq_ema_update: publish a contiguous f32 tensor of <= {mb.floats} values")
        seq, slot = res = mb.reserve()
        c.pub_src, c.pub_n, c.pub_copy, c.pub_box = ptr(src), src.numel(), ptr(copy), mb._dev
        c.pub_slot, c.pub_slots, c.pub_floats, c.pub_seq = slot, mb.slots, mb.floats, seq
    if rows is not None:
        src, idx = rows
        _check_cuda(src)
        if idx.dtype != torch.int32 or idx.is_cuda or idx.numel() != K or not idx.is_contiguous() or src.shape[1] != D:
            raise ValueError("vq_ema_update: rows = (src [n, D] device, K host int32 indices)")
        c.rows_src, c.rows_ld, c.n_rows, c.rows_host = ptr(src), src.stride(0), K, idx.data_ptr()
    call("vqx_vq_ema_update_close", ptr(emb_sum), ptr(emb_elem), ptr(E), ptr(bsum), ptr(bcnt), ptr(rand_rows), K, D,
         mu, threshold, ptr(diag), ptr(partials), ctypes.addressof(c), stream_ptr())
    return res


def gather_rows(src, rows, out):
    call("vqx_gather_rows", ptr(src), src.stride(0), ptr(rows), out.shape[0], out.shape[1], ptr(out), stream_ptr())
    return out


def gather_rows_host(src, rows, out):
    """out[i] = src[rows[i]] (zero rows for negative ids) with `rows` a host
    int32 tensor passed to the kernels by value (no copy on the stream)."""
    _check_cuda(src, out)
    if rows.device.type != "cpu" or rows.numel() != out.shape[0]:
        raise ValueError("gather_rows_host: rows must be a host tensor of out.shape[0] ids")
    if not out.is_contiguous() or out.dim() != 2 or out.shape[1] > src.shape[1] or src.stride(1) != 1:
        raise ValueError("gather_rows_host: out must be contiguous [n, D] with D <= src's row width")
    if rows.numel() and (int(rows.max()) >= src.shape[0] or int(rows.min()) < -1):
        raise ValueError(f"gather_rows_host: row ids must lie in [-1, {src.shape[0]})")
    rows = rows.to(torch.int32).contiguous()
    call("vqx_gather_rows_host", ptr(src), src.stride(0), rows.data_ptr(), out.shape[0], out.shape[1], ptr(out),
         stream_ptr())
    return out


def vq_commit_bwd(z, zq, scale, dz):
    call("vqx_vq_commit_bwd", ptr(z), ptr(zq), z.numel(), scale, ptr(dz), dt_code(dz.dtype), stream_ptr())
    return dz


COMMIT_PARTS = 256  # vqx.h VQX_COMMIT_PARTS


def vq_commit_bwd_cs(z, zq, scale, dz, partials):
    """vq_commit_bwd plus partials[p][d] = column sums of the stored dz over row part p
    (COMMIT_PARTS parts; the first level of the bias gradient of the conv producing z)."""
    _check_cuda(z, zq, dz, partials)
    N, D = z.shape
    if tuple(partials.shape) != (COMMIT_PARTS, D) or not partials.is_contiguous() or tuple(dz.shape) != (N, D) \
            or not (z.is_contiguous() and zq.is_contiguous() and dz.is_contiguous()):
        raise ValueError("vq_commit_bwd_cs: contiguous z/zq/dz [N, D] and partials [COMMIT_PARTS, D] expected")
    call("vqx_vq_commit_bwd_cs", ptr(z), ptr(zq), N, D, scale, ptr(dz), dt_code(dz.dtype), ptr(partials),
         stream_ptr())
    return dz


def time_gather(x, y, B, T, src_t):
    call("vqx_time_gather", ptr(x), ptr(y), B, T, x.shape[1], ptr(src_t), dt_code(x.dtype), stream_ptr())
    return y


def embedding_fwd(weight, ids, out):
    call("vqx_embedding_fwd", ptr(weight), ptr(ids), ids.numel(), weight.shape[1], ptr(out), stream_ptr())
    return out


def embedding_bwd(dout, ids, dweight):
    call("vqx_embedding_bwd", ptr(dout), ptr(ids), ids.numel(), dweight.shape[1], ptr(dweight), stream_ptr())
    return dweight


def embedding_bwd_rows(dout, ids, dweight, accumulate=False):
    """Every row of dweight: (+)= the sum of dout's rows whose id is that row, in
    batch order (0 where absent); no zero fill needed before it."""
    _check_cuda(dout, ids, dweight)
    if ids.dtype != torch.int64 or not (dout.is_contiguous() and dweight.is_contiguous()):
        raise ValueError("embedding_bwd_rows: int64 ids, contiguous dout / dweight")
    _span(dout, ids.numel() * dweight.shape[1], "embedding dout")
    _span(ids, ids.numel(), "embedding ids")
    call("vqx_embedding_bwd_rows", ptr(dout), ptr(ids), ids.numel(), dweight.shape[1], dweight.shape[0], ptr(dweight),
         int(accumulate), stream_ptr())
    return dweight


def linear_f32(c, W, bias, out):
    B, I = c.shape
    O = W.shape[0]
    call("vqx_linear_f32", ptr(c), ptr(W), ptr(bias), B, I, O, ptr(out), stream_ptr())
    return out


def linear_bwd_f32(dout, c, W, dW=None, dc=None):
    B, I = c.shape
    O = W.shape[0]
    call("vqx_linear_bwd_f32", ptr(dout), ptr(c), ptr(W), B, I, O, ptr(dW), ptr(dc), stream_ptr())


def grad_sq_norm(g, partials, out):
    call("vqx_grad_sq_norm", ptr(g), g.numel(), ptr(partials), ptr(out), stream_ptr())
    return out


def adam_hyper(step, lr0, gamma, step_size, beta1, beta2, eps, hyper):
    call("vqx_adam_hyper", ptr(step), lr0, gamma, step_size, beta1, beta2, eps, ptr(hyper), stream_ptr())


def adam_step(p, g, m, v, hyper, sumsq, max_norm):
    call("vqx_adam_step", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), ptr(hyper), ptr(sumsq), max_norm,
         stream_ptr())


def radam_hyper(step, lr0, gamma, step_size, beta1, beta2, eps, hyper):
    call("vqx_radam_hyper", ptr(step), lr0, gamma, step_size, beta1, beta2, eps, ptr(hyper), stream_ptr())


def adam_step_wn(p, g, m, v, hyper, sumsq, max_norm, rows_table, segs):
    """adam_step plus the next forward's weight-norm preparation of the rows
    in `rows_table` (wn_table of weight-normed convs); `segs` = (host int64
    [n, 2] tensor, its device copy) of the other flat ranges."""
    arr, dev = rows_table
    sh, sd = segs
    call("vqx_adam_step_wn", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), ptr(hyper), ptr(sumsq), max_norm,
         ctypes.addressof(arr), dev.data_ptr(), len(arr), sh.data_ptr() if sh.numel() else None,
         ptr(sd) if sh.numel() else None, sh.shape[0], stream_ptr())


def radam_step(p, g, m, v, hyper, sumsq, max_norm):
    call("vqx_radam_step", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), ptr(hyper), ptr(sumsq), max_norm,
         stream_ptr())


def convert_2d(src, dst, rows=None, cols=None):
    """dst[:rows, :cols] = src (dtype-converting, strided); src=None zero-fills."""
    rows = dst.shape[0] if rows is None else rows
    cols = dst.shape[1] if cols is None else cols
    call("vqx_convert_2d", ptr(src), src.stride(0) if src is not None else 0,
         dt_code(src.dtype) if src is not None else 0, ptr(dst), dst.stride(0), dt_code(dst.dtype), rows, cols,
         stream_ptr())
    return dst


def convert_2d_zero2(src, dst, zero_dst):
    """dst = src (dtype-converting, strided) and zero_dst = 0 (dst's dtype), one launch."""
    _check_cuda(src, dst, zero_dst)
    if tuple(src.shape) != tuple(dst.shape) or zero_dst.dtype != dst.dtype or zero_dst.dim() != 2:
        raise ValueError("convert_2d_zero2: src and dst must share a shape, zero_dst dst's dtype")
    call("vqx_convert_2d_zero2", ptr(src), src.stride(0), dt_code(src.dtype), ptr(dst), dst.stride(0),
         dt_code(dst.dtype), dst.shape[0], dst.shape[1], ptr(zero_dst), zero_dst.stride(0), zero_dst.shape[0],
         zero_dst.shape[1], stream_ptr())
    return dst


def zero_(t):
    """Zero a contiguous f32/bf16 device tensor with the native fill."""
    flat = t.view(1, -1)
    return convert_2d(None, flat)


def scale_act_2d(src, dst, scale, act, rows=None, cols=None):
    """dst = act(scale * src) (strided, dtype-converting)."""
    rows = dst.shape[0] if rows is None else rows
    cols = dst.shape[1] if cols is None else cols
    call("vqx_scale_act_2d", ptr(src), src.stride(0), dt_code(src.dtype), ptr(dst), dst.stride(0), dt_code(dst.dtype),
         rows, cols, scale, act, stream_ptr())
    return dst


def vq_normalize(z, E, z_norm, z_len, emb_norm, e_len, partials, normloss_out=None):
    """embed_norm() in place on E, emb_norm = E/||E||, z_norm = z/||z|| (+ sum (z_norm - z)^2)."""
    call("vqx_vq_normalize", ptr(z), z.shape[0], z.shape[1], ptr(E), E.shape[0], ptr(z_norm), ptr(z_len),
         ptr(emb_norm), ptr(e_len), ptr(partials), ptr(normloss_out), stream_ptr())


def vq_perplexity(counts, n_rows, out):
    call("vqx_vq_perplexity", ptr(counts), counts.shape[0], n_rows, ptr(out), stream_ptr())


def vq_plain_bwd(z, z_norm, z_len, zq, dzq, src_t, T, normalize, beta, scale, dz, bsum, bcnt, emb, e_len, dE):
    call("vqx_vq_plain_bwd", ptr(z), ptr(z_norm), ptr(z_len), ptr(zq), ptr(dzq), ptr(src_t), T, zq.shape[0],
         zq.shape[1], int(normalize), beta, scale, ptr(dz), dt_code(dz.dtype), ptr(bsum), ptr(bcnt), ptr(emb),
         ptr(e_len), emb.shape[0], ptr(dE), stream_ptr())


def cu_masked_stream(reserve_cus):
    """A torch ExternalStream on all but `reserve_cus` CUs of the current
    device (vqx_stream_create_cu_mask) and the CU count it may use; release it
    with release_stream(stream)."""
    s = ctypes.c_void_p()
    used = ctypes.c_int32()
    call("vqx_stream_create_cu_mask", int(reserve_cus), ctypes.byref(s), ctypes.byref(used))
    return torch.cuda.ExternalStream(s.value), used.value


def release_stream(stream):
    call("vqx_stream_destroy", ctypes.c_void_p(stream.cuda_stream))


class Mailbox:
    """Host mailbox for small per-step statistics (vqx_mailbox_*): `slots`
    slots of `floats` f32 values in mapped pinned host memory, each with a
    sequence number the publishing kernel stores last (system-scope release).
    publish() enqueues the copy on the current stream; read(seq, slot) polls
    the slot's number on the host -- no event, no copy on the stream."""

    def __init__(self, slots=64, floats=16):
        import numpy as np
        self.slots, self.floats = int(slots), int(floats)
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        call("vqx_mailbox_create", self.slots, self.floats, ctypes.byref(h), ctypes.byref(d))
        self._host, self._dev = h.value, d.value
        n = self.slots + self.slots * self.floats
        buf = (ctypes.c_uint32 * n).from_address(self._host)
        self._seq = np.frombuffer(buf, dtype=np.uint32, count=self.slots)
        self._val = np.frombuffer(buf, dtype=np.float32, count=self.slots * self.floats,
                                  offset=4 * self.slots).reshape(self.slots, self.floats)
        self._next = 1

    def publish(self, src, dev_copy=None):
        """Publish src (f32 device tensor, <= floats values) as the next
        sequence number; returns (seq, slot)."""
        _check_cuda(src, dev_copy)
        n = src.numel()
        if n > self.floats or not src.is_contiguous() or src.dtype != torch.float32:
            raise ValueError(f"Mailbox.publish: contiguous f32 tensor of <= {self.floats} values")
        seq, slot = self.reserve()
        call("vqx_mailbox_publish", ptr(src), n, ptr(dev_copy), self._dev, slot, self.slots, self.floats, seq,
             stream_ptr())
        return seq, slot

    def reserve(self):
        """The next (seq, slot), for a launch that publishes itself
        (vq_ema_update(publish=...))."""
        seq, self._next = self._next, self._next + 1
        return seq, seq % self.slots

    def try_read(self, seq, slot, n):
        """The values of `seq` once published (None while pending); raises
        LookupError when the slot has been reused by a later step."""
        s = int(self._seq[slot])
        if s < seq:
            return None
        if s > seq:
            raise LookupError("mailbox slot reused")
        v = self._val[slot, :n].copy()
        if int(self._seq[slot]) != seq:  # overwritten while copying
            raise LookupError("mailbox slot reused")
        return v

    def __del__(self):
        try:
            if getattr(self, "_host", None):
                L.load().vqx_mailbox_destroy(ctypes.c_void_p(self._host))
                self._host = None
        except Exception:
            pass
