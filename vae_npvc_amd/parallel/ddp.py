"""Data parallelism for the VQ-VAE step: one process per GPU, torch.distributed
over RCCL (backend "nccl" on ROCm) across the node's xGMI links.

Per step:
  * gradients — the flat fp32 gradient buffer follows model.parameters()
    order (encoder first; each backward layer group's parameters -- weights,
    biases, GroupNorm affine -- are contiguous in it) and is all-reduced
    (mean) run by run as soon as a run is final: the engine tracks which
    parameters each backward group's weight-norm + column-reduction launch
    finalises and launches the maximal contiguous ready runs (>= 64 K floats,
    split into buckets of BUCKET_BYTES) asynchronously, so the reduction
    overlaps the rest of the backward whatever order the groups finish in
    (engine/step.py `_grads_final`).  Mean over ranks
    of per-rank frame_mean losses equals the global-batch loss, so clipping
    after the reduce is identical on all ranks.
  * EMA statistics — bsum [K, D], bcnt [K] and the dead-code rows are summed
    in ONE all-reduce right after the VQ kernel; it overlaps the decoder and
    the backward (the codebook update runs at the end of the step).  Every
    rank draws the same CPU randperm(N_global); each fills the rows it owns,
    so the sum assembles exactly the global batch's z[perm[:K]].
No other collective sits on the data path.

Comm(overlap=False) (config `grad_sync: end`, bench.py --grad-sync end) holds
the gradient runs back and issues them all in finish(), after the backward:
RCCL's device kernel (248-256 VGPRs on gfx950) takes a GEMM workgroup slot on
every CU it occupies, and the one-round GEMM grids lose 20-25% while it is
resident (profiles/r04/cu_reserve.txt), so the switch trades that for the
all-reduce's own time on the critical path.
"""
import torch
import torch.distributed as dist

BUCKET_BYTES = 64 << 20  # ~16M fp32 gradients per all-reduce (per-link ring ≈ 0.5 ms at 8 GPUs)


def owned_rows(perm, rank_offset, n_local):
    """Map global row ids (a randperm of the global batch's frames) to this
    rank's local rows; rows another rank owns become -1 (gathered as zeros),
    so a SUM all-reduce of the per-rank gathers assembles z_global[perm]."""
    loc = perm - rank_offset
    return torch.where((loc >= 0) & (loc < n_local), loc, torch.full_like(loc, -1))


class Comm:
    def __init__(self, group=None, bucket_bytes=BUCKET_BYTES, overlap=True):
        self.group = group
        self.overlap = overlap  # False: gradient runs all-reduced in finish(), after the backward
        self.held = []          # (lo, hi) runs held back when not overlapping
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = dist.get_backend(group)
        self.bucket = max(1, bucket_bytes // 4)
        self.pending = []
        # diagnostics (bench.py): bytes all-reduced, collectives issued and,
        # when `timing` is on, the time the compute stream stood still behind
        # the gradient / EMA all-reduces (event pairs around each wait)
        self.bytes = 0
        self.calls = 0
        self.timing = False
        self._waits = {"grad": [], "ema": []}

    def _account(self, t):
        self.bytes += t.numel() * t.element_size()
        self.calls += 1

    def wait(self, work, tag):
        """work.wait() on the current stream; timed under `timing` (RCCL: the
        compute stream's stall until the collective has finished)."""
        if not (self.timing and self.backend == "nccl"):
            work.wait()
            return
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        work.wait()
        e1.record()
        self._waits[tag].append((e0, e1))

    def reset_stats(self):
        self.bytes = self.calls = 0
        self._waits = {"grad": [], "ema": []}

    def stats(self):
        """(bytes, collectives, grad-wait ms, EMA-wait ms) since reset_stats();
        synchronises on the recorded events."""
        ms = {k: sum(a.elapsed_time(b) for a, b in v) for k, v in self._waits.items()}
        return self.bytes, self.calls, ms["grad"], ms["ema"]

    def _avg_op(self):
        return dist.ReduceOp.AVG if self.backend == "nccl" else dist.ReduceOp.SUM

    def all_reduce_sum(self, t, async_op=False):
        self._account(t)
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)

    def all_gather_cat(self, t):
        """Concatenation over ranks (rank order) of a per-rank tensor; gloo
        gathers through host memory."""
        src = t.contiguous() if self.backend == "nccl" else t.detach().cpu()
        parts = [torch.empty_like(src) for _ in range(self.world)]
        dist.all_gather(parts, src, group=self.group)
        return torch.cat(parts).to(t.device)

    def grads_ready(self, flat, lo, hi):
        """Launch async mean all-reduces over flat[lo:hi] in buckets (held
        until finish() when not overlapping)."""
        if not self.overlap:
            self.held.append((flat, lo, hi))
            return
        self._launch(flat, lo, hi)

    def _launch(self, flat, lo, hi):
        op = self._avg_op()
        for s in range(lo, hi, self.bucket):
            view = flat[s: min(hi, s + self.bucket)]
            self._account(view)
            work = dist.all_reduce(view, op=op, group=self.group, async_op=True)
            self.pending.append((work, view))

    def finish(self):
        """Make the current stream wait for every launched reduce (first
        launching the held runs, adjacent ones merged, when not overlapping)."""
        if self.held:
            runs = sorted(self.held, key=lambda r: r[1])
            self.held = []
            flat, lo, hi = runs[0]
            for f, a, b in runs[1:]:
                if f is flat and a == hi:
                    hi = b
                    continue
                self._launch(flat, lo, hi)
                flat, lo, hi = f, a, b
            self._launch(flat, lo, hi)
        timed = self.timing and self.backend == "nccl" and self.pending
        if timed:  # one event pair around all the waits: the stream's total stall
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        for work, view in self.pending:
            work.wait()
            if self.backend != "nccl":
                view.div_(self.world)
        if timed:
            e1.record()
            self._waits["grad"].append((e0, e1))
        self.pending = []

    def mean_scalars(self, t):
        dist.all_reduce(t, op=self._avg_op(), group=self.group)
        if self.backend != "nccl":
            t.div_(self.world)
        return t
