"""Out-of-extent write detection for the engine's buffers (a debugging mode,
EngineOptions.debug_checks; off in every measured run).

Two layers:
  * guard canaries -- every buffer the engine allocates (activations, split-K
    slab arena, flat parameter / gradient / Adam buffers, packed weights,
    statistics, the quantizer's EMA buffers) is carved out of a larger
    allocation with GUARD bytes of a fixed pattern before and after it.  After
    every libvqx entry point (_lib.call's post-call hook) the stream is
    synchronised and every guard is compared with the pattern in one pass; a
    changed byte names the entry point that wrote it and the buffer whose
    extent it overran;
  * host extent checks (ops.py, `ops.set_debug_checks`): before a call, the
    span each pointer argument will be read or written over (rows, leading
    dimension, columns, split-K slabs, partial-sum tiles) is compared with the
    tensor's storage, so a mis-sized argument raises before any kernel runs.

Used by tests/test_gpu_config3.py's audit of the 8-rank step (VERDICT r05
item 1) and tests/test_gpu_kernels.py's self-test of the detector.
"""
import torch

from . import _lib as L
from . import ops

GUARD = 4096          # bytes each side (a multiple of 256 keeps every buffer 256-B aligned)
PATTERN = 0xA5


class GuardSet:
    """Guarded allocations of one engine and the check over all of them."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.guards = []   # (uint8 guard view, buffer label, "head" | "tail")
        self.raws = []     # the guarded allocations (kept alive: their pointers stay unique)
        self.calls = 0
        self.checks = 0

    def empty(self, *shape, dtype=torch.float32, label="buffer"):
        if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)):
            shape = tuple(shape[0])
        n = 1
        for s in shape:
            n *= int(s)
        esz = torch.empty((), dtype=dtype).element_size()
        nbytes = n * esz
        raw = torch.empty(GUARD + nbytes + GUARD, device=self.device, dtype=torch.uint8)
        raw.fill_(PATTERN)
        ops._logical_end[raw.untyped_storage().data_ptr()] = GUARD + nbytes  # host checks stop at the tail guard
        self.raws.append(raw)
        data = raw[GUARD:GUARD + nbytes].view(dtype).view(*shape) if shape else raw[GUARD:GUARD + nbytes].view(dtype)
        self.guards.append((raw[:GUARD], label, "head"))
        self.guards.append((raw[GUARD + nbytes:], label, "tail"))
        return data

    def zeros(self, *shape, dtype=torch.float32, label="buffer"):
        t = self.empty(*shape, dtype=dtype, label=label)
        t.zero_()
        return t

    def adopt(self, t, label):
        """A guarded copy of an existing tensor (module buffers the kernels write)."""
        g = self.empty(*t.shape, dtype=t.dtype, label=label)
        g.copy_(t)
        return g

    def check(self, where):
        """Synchronise and compare every guard with the pattern; raise naming
        `where` (the entry point that just ran) and the overrun buffers."""
        self.checks += 1
        if not self.guards:
            return
        torch.cuda.synchronize(self.device)
        flat = torch.cat([g for g, _, _ in self.guards])
        bad = flat != PATTERN
        if not bool(bad.any()):
            return
        hits, o = [], 0
        for g, label, side in self.guards:
            n = g.numel()
            b = bad[o:o + n]
            if bool(b.any()):
                first = int(torch.nonzero(b)[0])
                hits.append(f"{label} ({side} guard: {int(b.sum())} bytes changed, first at +{first})")
                g.fill_(PATTERN)  # report each overrun once
            o += n
        raise AssertionError(f"out-of-extent write after {where}: " + "; ".join(hits))


_active = []


def install(gs):
    """Check `gs` after every libvqx entry point of this process."""
    _active.append(gs)
    L.set_post_call(_post_call)


def uninstall(gs):
    """Stop checking `gs` (and forget its extents)."""
    if gs in _active:
        _active.remove(gs)
    for raw in gs.raws:
        ops._logical_end.pop(raw.untyped_storage().data_ptr(), None)
    if not _active:
        L.set_post_call(None)
        ops.set_debug_checks(False)


_PURE = {"vqx_colsum_parts", "vqx_vq_workspace", "vqx_wgrad_tiles", "vqx_weight_norm_bwd_partials", "vqx_version",
         "vqx_last_error", "vqx_probe_enable", "vqx_probe_select", "vqx_probe_clear", "vqx_probe_count",
         "vqx_probe_read"}


def _post_call(name):
    if name in _PURE:
        return
    for gs in list(_active):
        gs.calls += 1
        gs.check(name)
