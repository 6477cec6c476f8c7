"""The VQ forward's fast path (vqx_vq.hip vq_fast_kernel + vq_fix_kernel:
fp16 MFMA distances, each frame's argmin certified against a rigorous bound on
the difference to the fp32 distances, uncertified frames re-ranked exactly)
against the fp32 MFMA kernel (vqx_vq_set_path(1)): indices, z_q and the
decoder copy bit for bit, the commitment sum to fp32 rounding (per-frame
terms, another summation order).  Inputs that exercise every branch: codebooks
drawn from the frames (the trained regime: certified), random codebooks,
duplicated codes (exact ties: the lowest index wins), codes perturbed in the
last bits (ties closer than the bound: re-ranked), magnitudes beyond the fp16
range (every frame re-ranked), NaN frames, ragged N and K from 16 to 512."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(z, E, path):
    from vae_npvc_amd import _lib as L, ops
    N, K = z.shape[0], E.shape[0]
    idx = torch.full((N,), -7, dtype=torch.int64, device=DEV)
    zq = torch.full((N, 128), float("nan"), device=DEV)
    zqc = torch.full((N, 128), float("nan"), device=DEV, dtype=torch.bfloat16)
    sq = torch.zeros(1, device=DEV)
    part = torch.empty(ops.vq_workspace(N, K, False), device=DEV)
    L.call("vqx_vq_set_path", path)
    try:
        ops.vq_forward(z, E, idx, zq, zqc, sq, part, None, None)
        torch.cuda.synchronize()
    finally:
        L.call("vqx_vq_set_path", 0)
    return idx, zq, zqc, sq


def _case(kind, N, K, seed):
    g = torch.Generator().manual_seed(seed)
    z = torch.randn(N, 128, generator=g) * 2.0
    if kind == "rows":          # codebook = frames (init_emb): well separated
        E = z[torch.randperm(N, generator=g)[:K]].clone()
    elif kind == "randn":
        E = torch.randn(K, 128, generator=g) * 2.0
    elif kind == "dups":        # exact duplicates of one code at several indices + frames equal to codes
        E = torch.randn(K, 128, generator=g)
        E[K // 2] = E[3]
        E[K - 1] = E[3]
        z[:K // 4] = E[torch.randint(0, K, (K // 4,), generator=g)]
    elif kind == "near":        # codes 1-2 ulp apart: ties below the bound, re-ranked exactly
        base = torch.randn(K // 8, 128, generator=g)
        E = base.repeat(8, 1)
        E = E + torch.randint(-2, 3, E.shape, generator=g) * E.abs() * 2.0 ** -23
        z = base[torch.randint(0, K // 8, (N,), generator=g)] + torch.randn(N, 128, generator=g) * 1e-3
    elif kind == "huge":        # beyond the fp16 range: every frame goes to the exact re-rank
        E = torch.randn(K, 128, generator=g) * 4e4
        z = z * 2e4
    elif kind == "nan":
        E = torch.randn(K, 128, generator=g)
        z[5] = float("nan")
        z[N - 1, 7] = float("nan")
    return z.to(DEV).contiguous(), E.to(DEV).contiguous()


@pytest.mark.parametrize("kind,N,K", [("rows", 16384, 512), ("randn", 16384, 512), ("rows", 4000, 128),
                                      ("randn", 777, 16), ("dups", 3000, 512), ("near", 2048, 256),
                                      ("near", 5000, 512), ("huge", 1000, 64), ("nan", 1000, 128),
                                      ("randn", 65, 512)])
def test_fast_vq_path_equals_fp32_kernel(kind, N, K):
    z, E = _case(kind, N, K, 3)
    ref = _run(z, E, 1)
    got = _run(z, E, 0)
    assert torch.equal(ref[0], got[0]), (kind, int((ref[0] != got[0]).sum()))
    assert torch.equal(ref[1].view(torch.int32), got[1].view(torch.int32))
    assert torch.equal(ref[2].view(torch.int16), got[2].view(torch.int16))
    a, b = ref[3].item(), got[3].item()
    if kind == "nan":
        assert a != a and b != b
    else:
        assert abs(a - b) <= 1e-5 * abs(a) + 1e-30, (a, b)
