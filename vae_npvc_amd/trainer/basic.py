"""Drop-in Trainer for `trainer_type: vae_npvc_amd.trainer.basic` (the
reference's seam, vae_npvc/bin/train.py:33,49-51).  Same surface as
vae_npvc/trainer/basic.py:10-121 — Trainer(config), train_step(input,
iteration=None) -> (iteration, loss_detail), valid, valid_step,
get_model_info, save_checkpoint, load_checkpoint — with the step fused on the
MI355X: forward, backward, global-norm clip, Adam or RAdam (betas
(0.5, 0.999), wd 0, trainer/basic.py:30-39) and StepLR run as HIP kernels
with no host synchronisation; the optimizer state is saved in the
torch.optim.Adam / reference RAdam state_dict format so reference checkpoints
({'model', 'optimizer', 'iteration'}) load both ways.

Data parallel: when torch.distributed is initialised, each rank trains on its
own shard (per-rank batch) and the engine all-reduces gradients and EMA
statistics (vae_npvc_amd/parallel/ddp.py).
"""
from collections.abc import Mapping
from importlib import import_module

import torch
import torch.distributed as dist

from .. import ops


class LazyLossDetail(Mapping):
    """loss_detail dict of one step (instead of the reference's 7 .item()
    syncs, vqvae.py:85-87 and layers_vq.py:229-232).  The step's statistics
    are snapshotted on the device by a kernel (the next step overwrites
    them) and copied to the host only when a value is first read.  An eager
    asynchronous D2H per step (EngineOptions.lazy_stats false) held the
    compute stream ~10 us after the runtime copy even when nothing read the
    values.

    Round 6: every statistic is final at the end of the forward (the EMA
    update runs there, where the reference runs it, layers_vq.py:295-296), so
    the engine publishes them right after the log-loss launch into a host
    mailbox (ops.Mailbox: mapped pinned memory, a sequence number stored
    behind a system-scope release; VQVAEEngine.forward_train).  A read polls
    that number, so it waits for the forward, not for the backward and
    optimizer queued behind it: a loop that reads every step (the reference's
    bin/train.py:128-132) enqueues the next step while the GPU still runs
    this one's backward.  No event or copy enters the stream."""

    def __init__(self, engine, w, stats_dev):
        self._eng, self._w = engine, w
        self._d = None
        self._ev = None
        pub = getattr(w, "stats_snap", None)
        self._pub = None
        if engine.opt.lazy_stats and pub is not None:
            self._pub = pub          # published mid-step into the engine's host mailbox
            w.stats_snap = None
            self._snap = self._snap_ev = self._host = None
        elif engine.opt.lazy_stats:
            self._snap, self._snap_ev = torch.empty_like(stats_dev), None
            ops.convert_2d(stats_dev.view(1, -1), self._snap.view(1, -1))
            self._host = None
        else:
            self._snap = self._snap_ev = None
            self._host = torch.empty(stats_dev.shape, dtype=stats_dev.dtype, pin_memory=True)
            self._host.copy_(stats_dev, non_blocking=True)
            self._ev = torch.cuda.Event()
            self._ev.record()

    def _read_mailbox(self):
        """Poll the mailbox slot until the step's values are there; a slot
        already reused by a later step, or a stream that has finished without
        the values arriving, falls back to the device copy."""
        mb, seq, slot, snap, stream = self._pub
        self._pub = None
        spins = 0
        while True:
            try:
                v = mb.try_read(seq, slot, snap.numel())
            except LookupError:
                return snap.cpu()
            if v is not None:
                return torch.from_numpy(v)
            spins += 1
            if spins % 4096 == 0 and stream.query():  # the stream finished: one last look, then the copy
                try:
                    v = mb.try_read(seq, slot, snap.numel())
                except LookupError:
                    v = None
                return torch.from_numpy(v) if v is not None else snap.cpu()

    def _get(self):
        if self._d is None:
            if self._pub is not None:
                host = self._read_mailbox()
            elif self._snap is not None:
                host = self._snap.cpu()
                self._snap = None
            else:
                self._ev.synchronize()
                host = self._host
            self._d = self._eng.loss_detail(self._w, host)
        return self._d

    def __getitem__(self, k):
        return self._get()[k]

    def __iter__(self):
        return iter(self._get())

    def __len__(self):
        return len(self._get())

    def __repr__(self):
        return repr(self._get())


class FusedOptimState:
    """state_dict view over the engine's flat moments in the format of
    torch.optim.Adam (optim_type Adam) or of the reference's RAdam
    (trainer/radam.py:30-33: step as a Python int, no Adam-only group keys)."""

    def __init__(self, trainer):
        self.t = trainer

    def _lr_now(self, step):
        e = self.t.engine
        return e.lr0 * (e.sched_gamma ** ((max(step, 1) - 1) // e.sched_step)) if step else e.lr0

    def state_dict(self):
        e = self.t.engine
        step = int(e.opt_step.item())
        state = {}
        off = 0
        for i, p in enumerate(e.params):
            n = p.numel()
            if step > 0:
                state[i] = {"step": torch.tensor(float(step)) if e.opt_kind == "adam" else step,
                            "exp_avg": e.exp_avg[off:off + n].view_as(p).detach().cpu().clone(),
                            "exp_avg_sq": e.exp_avg_sq[off:off + n].view_as(p).detach().cpu().clone()}
            off += n
        group = {"lr": self._lr_now(step + 1), "betas": tuple(e.betas), "eps": e.eps, "weight_decay": 0.0}
        if e.opt_kind == "adam":
            group.update({"amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
                          "differentiable": False, "fused": None})
        group["params"] = list(range(len(e.params)))
        if self.t.scheduler_cfg is not None:
            group["initial_lr"] = e.lr0
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd):
        e = self.t.engine
        st = sd["state"]
        off = 0
        step = 0
        with torch.no_grad():
            for i, p in enumerate(e.params):
                n = p.numel()
                s = st.get(i, st.get(str(i)))
                if s is not None:
                    e.exp_avg[off:off + n].copy_(s["exp_avg"].reshape(-1).to(e.device))
                    e.exp_avg_sq[off:off + n].copy_(s["exp_avg_sq"].reshape(-1).to(e.device))
                    step = int(float(s["step"]))
                off += n
            e.opt_step.fill_(step)


class Trainer(object):
    def __init__(self, config):
        model_type = config.get("model_type", "vae_npvc_amd.model.vqvae:Model").split(":")
        self.learning_rate = config.get("learning_rate", 1e-3)
        self.max_grad_norm = config.get("max_grad_norm", 5)
        optim_type = str(config.get("optim_type", "Adam"))
        self.optim_kind = "radam" if optim_type.upper() == "RADAM" else "adam"  # trainer/basic.py:30-39
        lr_sched = config.get("lr_scheduler", None)
        lr_param = config.get("lr_param", {"step_size": 100000, "gamma": 0.5, "last_epoch": -1})
        self.scheduler_cfg = lr_param if lr_sched is not None else None
        # gradient all-reduce beside the backward ("overlap") or after it ("end"); parallel/ddp.py
        self.grad_sync = str(config.get("grad_sync", "overlap"))
        if self.grad_sync not in ("overlap", "end"):
            raise ValueError(f"grad_sync must be 'overlap' or 'end', not {self.grad_sync!r}")
        # load_checkpoint restores the iteration counter (a resumed run continues at
        # checkpoint + 1).  The reference's load_checkpoint returns the checkpoint's
        # iteration without restoring its counter (trainer/basic.py:117-121), so its
        # first train_step after a resume returns 1 and bin/train.py's loop restarts
        # counting there; `reference_resume_counter: true` keeps that behaviour.
        self.reference_resume_counter = bool(config.get("reference_resume_counter", False))

        module = import_module(model_type[0], package=None)
        model_name = "Model" if len(model_type) < 2 else model_type[1]
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.model = getattr(module, model_name)(config).to(self.device)
        self.model.train()
        self._setup_engine()
        self.optimizer = FusedOptimState(self)
        self.scheduler = None  # StepLR runs on the device inside the Adam kernel's hyper-parameter step
        self.iteration = 0

    def _setup_engine(self):
        """(Re)build the fused engine over the model's current parameters:
        data-parallel wiring, identical initial weights on every rank, fresh
        optimizer moments."""
        self.engine = self.model.engine(self.device)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            from ..parallel.ddp import Comm
            self.engine.attach_comm(Comm(overlap=self.grad_sync == "overlap"))
            dist.broadcast(self.engine.flat_p, 0)
            for b in self.model.buffers():
                dist.broadcast(b, 0)
            self.engine.invalidate_packed()  # the parameters were rewritten outside the fused Adam
        sp = self.scheduler_cfg or {}
        self.engine.init_optimizer(self.learning_rate, betas=(0.5, 0.999), eps=1e-8,
                                   max_grad_norm=float(self.max_grad_norm),
                                   sched_step=sp.get("step_size") if self.scheduler_cfg else None,
                                   sched_gamma=sp.get("gamma", 1.0) if self.scheduler_cfg else 1.0,
                                   kind=self.optim_kind)

    def train_step(self, input, iteration=None):
        if not self.model.training:
            raise RuntimeError("train_step needs the model in training mode (valid_step restores it; "
                               "call model.train() after a manual model.eval())")
        x, y = input
        x = x.to(self.device, non_blocking=True).float().contiguous()
        y = y.to(self.device, non_blocking=True)
        w = self.engine.train_step(x, y)
        # trainer/basic.py:74-77: the passed iteration is ignored and the
        # trainer's own counter advances (bin/train.py:126 feeds the returned
        # value back in).  The reference's iteration=None branch raises
        # (None + 1); here it counts the same way.  load_checkpoint restores
        # the counter, so a resumed run continues at checkpoint + 1 (unless
        # reference_resume_counter: the reference's restart at 1).
        self.iteration += 1
        return self.iteration, LazyLossDetail(self.engine, w, w.stats)

    def valid(self, data_loader):
        loss_detail = dict()
        for batch in data_loader:
            for key, val in self.valid_step(batch).items():
                loss_detail.setdefault(key, []).append(val)
        return loss_detail

    def valid_step(self, input):
        self.model.eval()
        with torch.no_grad():
            x, y = (t.to(self.device) for t in input)
            _, _, loss_detail = self.model((x, y))
        self.model.train()
        return loss_detail

    def get_model_info(self):
        return self.model

    def save_checkpoint(self, checkpoint_file):
        torch.save({"model": self.model.state_dict(), "optimizer": self.optimizer.state_dict(),
                    "iteration": self.iteration}, checkpoint_file)
        print("Saved state dict. to {}".format(checkpoint_file))

    def load_checkpoint(self, checkpoint_file):
        data = torch.load(checkpoint_file, map_location="cpu", weights_only=True)
        with torch.no_grad():
            self.model.load_state_dict(data["model"])
        if self.model._engine is not self.engine or not self.engine.params_intact():
            self._setup_engine()  # the codebook was resized (Model.load_state_dict, vqvae.py:106-119)
        self.optimizer.load_state_dict(data["optimizer"])
        if not self.reference_resume_counter:
            self.iteration = int(data["iteration"])
        return int(data["iteration"])
