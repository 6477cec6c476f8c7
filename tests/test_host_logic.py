"""Host-side logic of the drop-in path that runs without a GPU: the Jitter
neighbour map (numpy RNG stream), the StepLR learning-rate bookkeeping of the
fused optimizer state, and the data-parallel row-ownership mapping."""
import json
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from tests.helpers import GOLD


def engine_jitter_map(p, T):
    from vae_npvc_amd.engine.step import VQVAEEngine
    return VQVAEEngine.jitter_map(SimpleNamespace(dims={"jitter_p": p}), T)


def reference_semantics_map(p, T):
    """layers_vq.py:353-379 consuming numpy's global stream exactly as the
    reference does (np.random.choice per frame; replaces with prob. 1-p)."""
    src = np.arange(T)
    for i in range(T):
        replace = [True, False][np.random.choice([1, 0], p=[p, 1 - p])]
        if replace:
            if i == 0:
                src[i] = 1
            elif i == T - 1:
                src[i] = T - 2
            else:
                src[i] = i + np.random.choice([-1, 1], p=[0.5, 0.5])
    return src


@pytest.mark.parametrize("p", [0.0, 0.12, 0.5, 0.9])
@pytest.mark.parametrize("seed", [0, 7, 123])
def test_jitter_map_consumes_numpy_stream_like_reference(p, seed):
    np.random.seed(seed)
    want = reference_semantics_map(p, 300)
    tail_want = np.random.random_sample()
    np.random.seed(seed)
    got = engine_jitter_map(p, 300)
    tail_got = np.random.random_sample()
    assert np.array_equal(got, want)
    assert tail_got == tail_want  # same number of draws: later RNG users stay in sync


def test_jitter_map_matches_reference_golden():
    fx = json.load(open(GOLD / "jitter.json"))
    for v in fx.values():
        np.random.seed(v["seed"])
        assert engine_jitter_map(v["p"], v["T"]).tolist() == v["src"]


def test_step_lr_bookkeeping_matches_torch():
    """FusedOptimState reports the lr torch's Adam+StepLR would hold after `step`
    optimizer steps (trainer/basic.py:43-52 scheduler wiring)."""
    from vae_npvc_amd.trainer.basic import FusedOptimState
    lr0, gamma, size = 1e-3, 0.5, 3
    eng = SimpleNamespace(lr0=lr0, sched_gamma=gamma, sched_step=size)
    st = FusedOptimState(SimpleNamespace(engine=eng))
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.Adam([p], lr=lr0)
    sch = torch.optim.lr_scheduler.StepLR(opt, step_size=size, gamma=gamma)
    for step in range(12):
        # lr in effect for optimizer step `step + 1`
        assert st._lr_now(step + 1) == pytest.approx(opt.param_groups[0]["lr"], rel=1e-12)
        p.grad = torch.ones(1)
        opt.step()
        sch.step()


def test_owned_rows_partition_the_permutation():
    from vae_npvc_amd.parallel.ddp import owned_rows
    g = torch.Generator().manual_seed(3)
    n_local, world, K = 100, 4, 150
    perm = torch.randperm(n_local * world, generator=g)[:K]
    z = torch.randn(n_local * world, 5, generator=g)
    total = torch.zeros(K, 5)
    hits = torch.zeros(K, dtype=torch.int64)
    for r in range(world):
        loc = owned_rows(perm, r * n_local, n_local)
        mine = loc >= 0
        hits += mine.long()
        part = torch.zeros(K, 5)
        part[mine] = z[r * n_local:(r + 1) * n_local][loc[mine]]
        total += part
    assert torch.equal(hits, torch.ones(K, dtype=torch.int64))  # every row owned exactly once
    assert torch.equal(total, z[perm])  # the SUM all-reduce assembles z_global[perm]


def _loop_trainer(monkeypatch, start=0):
    """A Trainer whose device work is stubbed, to drive the host-side
    iteration contract on the CPU."""
    import vae_npvc_amd.trainer.basic as tb
    monkeypatch.setattr(tb, "LazyLossDetail", lambda eng, w, s: {"X like": 1.0})
    tr = tb.Trainer.__new__(tb.Trainer)
    tr.model = SimpleNamespace(training=True)
    tr.device = torch.device("cpu")
    tr.engine = SimpleNamespace(train_step=lambda x, y: SimpleNamespace(stats=None))
    tr.iteration = start
    return tr


def test_train_step_advances_under_reference_loop(monkeypatch):
    """bin/train.py:54,126 feeds the returned iteration back in
    (`iteration, d = trainer.train_step(batch, iteration=iteration)`); the
    reference Trainer ignores the argument and increments its own counter
    (trainer/basic.py:74-77), so the loop reaches max_iter."""
    tr = _loop_trainer(monkeypatch)
    batch = (torch.zeros(1, 2, 3), torch.zeros(1, 1, dtype=torch.int64))
    iteration, seen = 1, []
    while iteration <= 5:
        iteration, _ = tr.train_step(batch, iteration=iteration)
        seen.append(iteration)
    assert seen == [1, 2, 3, 4, 5, 6]
    # resume: load_checkpoint restores the counter, train.py passes ckpt + 1
    tr2 = _loop_trainer(monkeypatch, start=20)
    it, _ = tr2.train_step(batch, iteration=21)
    assert it == 21
    assert tr2.train_step(batch)[0] == 22  # iteration=None counts the same way


def test_resume_counter_restored_or_reference(monkeypatch, tmp_path):
    """load_checkpoint restores the iteration counter by default; with
    `reference_resume_counter` it only returns it, as the reference's
    (trainer/basic.py:117-121), whose next train_step then returns 1."""
    import vae_npvc_amd.trainer.basic as tb
    ckpt = tmp_path / "c.pt"
    torch.save({"model": {}, "optimizer": {}, "iteration": 40}, ckpt)
    batch = (torch.zeros(1, 2, 3), torch.zeros(1, 1, dtype=torch.int64))
    for ref_mode, expect in ((False, 41), (True, 1)):
        tr = _loop_trainer(monkeypatch)
        tr.engine = SimpleNamespace(train_step=lambda x, y: SimpleNamespace(stats=None), params_intact=lambda: True)
        tr.model = SimpleNamespace(training=True, load_state_dict=lambda sd: None, _engine=tr.engine)
        tr.optimizer = SimpleNamespace(load_state_dict=lambda sd: None)
        tr.reference_resume_counter = ref_mode
        assert tr.load_checkpoint(str(ckpt)) == 40
        assert tr.train_step(batch, iteration=41)[0] == expect


def test_load_state_dict_resizes_plain_codebook():
    """vqvae.py:106-119: a straight-through-VQ checkpoint with another codebook
    size rebuilds the quantizer at the checkpoint's shape and loads."""
    from tests.helpers import cfg_of
    from vae_npvc_amd.model.vqvae import Model
    cfg = cfg_of("vcc20", use_ema=False)
    src = Model(dict(cfg, z_num=256))
    sd = src.state_dict()
    m = Model(cfg)
    assert tuple(m.quantizer.embeddings.shape) == (512, 128)
    order = [k for k, _ in m.named_parameters()]
    m.load_state_dict(sd)
    assert tuple(m.quantizer.embeddings.shape) == (256, 128)
    assert torch.equal(m.quantizer.embeddings, sd["quantizer.embeddings"])
    assert m.quantizer.normalize == src.quantizer.normalize
    assert [k for k, _ in m.named_parameters()] == order  # parameter order kept (optimizer state lines up)


@pytest.mark.parametrize("name", ["vcc20", "vcc20_multi", "vcc20_nown", "vcc20_multi_nown"])
def test_model_parameters_match_reference_order(name):
    """Model(cfg) registers the reference's parameters in the reference's order
    (oracle.layer_specs, pinned by the reference-generated fixtures): with
    weight norm bias, weight_g, weight_v; with use_weight_norm false
    (vqvae.py:179-180,290-293) weight, bias -- on stride-1 and resampling convs."""
    from oracle.vqvae_cpu import layer_specs
    from tests.helpers import cfg_of
    from vae_npvc_amd.model.vqvae import Model
    cfg = cfg_of(name)
    m = Model(cfg)
    got = [(k, tuple(p.shape)) for k, p in m.named_parameters()]
    assert got == [(k, tuple(s)) for k, s in layer_specs(cfg)]
    if name.endswith("nown"):
        meta = json.load(open(GOLD / f"step_{name}.json"))
        assert [k for k, _ in got] == list(meta["params_after"])  # the reference's own parameter list


def test_remove_weight_norm_bakes_every_conv_including_resampling():
    """vqvae.py:93-103 on the general topology (stride-2 down-/up-sampling
    convs included): every weight-normed conv ends with a plain `weight`
    equal to g*v/||v|| (torch._weight_norm, dim 0) registered after `bias`,
    like torch.nn.utils.remove_weight_norm."""
    import torch
    from tests.helpers import cfg_of
    from vae_npvc_amd.model.resample import ResampleConv1d
    from vae_npvc_amd.model.vqvae import Model
    m = Model(cfg_of("vcc20_multi"))
    before = {n[: -len(".weight_v")]: torch._weight_norm(p, dict(m.named_parameters())[n[:-1] + "g"], 0).detach()
              for n, p in m.named_parameters() if n.endswith(".weight_v")}
    assert any(isinstance(x, ResampleConv1d) for x in m.modules())
    m.remove_weight_norm()
    names = [n for n, _ in m.named_parameters()]
    assert not any(n.endswith((".weight_g", ".weight_v")) for n in names)
    params = dict(m.named_parameters())
    for base, w in before.items():
        assert torch.equal(params[base + ".weight"], w), base
        assert names.index(base + ".weight") == names.index(base + ".bias") + 1


@pytest.mark.parametrize("name", ["vcc20_nown", "vcc20_multi_nown"])
def test_no_weight_norm_convs_get_kaiming_init(name):
    """use_weight_norm: false -- the reference's reset_parameters (vqvae.py:183,
    210-217, 296) re-draws every Conv1d / ConvTranspose1d weight with
    kaiming_normal_(nonlinearity='relu'): N(0, 2 / fan_in), torch's fan_in =
    weight.size(1) * kernel (for ConvTranspose1d that is cout * k).  The
    stride-1 and the resampling convs of both halves follow it; the biases keep
    the default uniform.  Statistical check on every weight of >= 4096 values:
    std within 8% of sqrt(2 / fan_in), mean within 4 standard errors of 0."""
    from tests.helpers import cfg_of
    from vae_npvc_amd.model.vqvae import Model
    torch.manual_seed(3)
    m = Model(cfg_of(name))
    checked = 0
    for n, p in m.named_parameters():
        if not n.endswith(".weight") or p.dim() != 3 or p.numel() < 4096:
            continue
        fan_in = p.size(1) * p.size(2)
        want = (2.0 / fan_in) ** 0.5
        std, mean = float(p.detach().std()), float(p.detach().mean())
        assert abs(std / want - 1) < 0.08, (n, std, want)
        assert abs(mean) < 4 * want / p.numel() ** 0.5, (n, mean)
        checked += 1
    assert checked >= 10, checked
    assert not any(n.endswith("weight_v") for n, _ in m.named_parameters())


def test_debug_extent_checks_refuse_short_buffers():
    """ops.set_debug_checks: a pointer argument whose buffer is shorter than the
    span the kernel would touch raises before any launch (host-side; CPU
    tensors suffice, no library call is made)."""
    from vae_npvc_amd import _lib as L
    from vae_npvc_amd import ops
    prev = ops.set_debug_checks(True)
    try:
        N, C = 256, 64
        x, w = torch.empty(N, C), torch.empty(C, 3 * C)
        ops.conv_args(x, w, torch.empty(N, C), T=128, cin=C, cout=C, ntaps=3, pad=1)  # exact sizes pass
        with pytest.raises(L.VqxError, match="conv y"):
            ops.conv_args(x, w, torch.empty(N - 1, C), T=128, cin=C, cout=C, ntaps=3, pad=1)
        with pytest.raises(L.VqxError, match="conv colsum_part"):
            ops.conv_args(x, w, torch.empty(N, C), T=128, cin=C, cout=C, ntaps=3, pad=1,
                          colsum=torch.empty(N // 128 - 1, C))
        big = torch.empty(N, 2 * C)  # a column view: its rows stride over the whole buffer
        ops.conv_args(x, w, big[:, C:], T=128, cin=C, cout=C, ntaps=3, pad=1)
        with pytest.raises(L.VqxError, match="conv y2"):
            ops.conv_args(x, w, big[:, :C], T=128, cin=C, cout=C, ntaps=3, pad=1, y2=big[1:, C:])
        with pytest.raises(L.VqxError, match="wgrad slabs"):
            ops.wgrad_args(x, x, torch.empty(4, C, 3 * C - 1), T=128, r_dim=C, c_dim=C, ntaps=3, pad=1, splits=4)
        # the guarded allocations' logical end (debug.py): the tail guard is not the buffer's
        raw = torch.empty(4096 + 4 * N + 4096, dtype=torch.uint8)
        ops._logical_end[raw.untyped_storage().data_ptr()] = 4096 + 4 * N
        try:
            t = raw[4096:4096 + 4 * N].view(torch.float32)
            ops._span(t, N, "guarded")
            with pytest.raises(L.VqxError, match="guarded"):
                ops._span(t, N + 1, "guarded")
        finally:
            ops._logical_end.pop(raw.untyped_storage().data_ptr(), None)
    finally:
        ops.set_debug_checks(prev)
    ops.conv_args(x, w, torch.empty(N - 1, C), T=128, cin=C, cout=C, ntaps=3, pad=1)  # off: no check
