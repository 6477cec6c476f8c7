"""Quantizer and jitter modules (buffers + API of vae_npvc/model/layers_vq.py).

The arithmetic (distance / argmin / gather / EMA update) is libvqx's fused HIP
kernels driven by the engine; these modules hold the state with the
reference's buffer names so checkpoints load both ways.
"""
import torch
import torch.nn as nn

from .. import ops


class EMAVectorQuantizer(nn.Module):
    """EMA codebook (layers_vq.py:166-334).  Buffers emb_init (bool),
    emb_sum [K, D], emb_elem [K], embeddings [K, D] (layers_vq.py:170-173)."""

    def __init__(self, z_num, z_dim, mu, threshold=1.0, reduction="frame_mean"):
        super().__init__()
        if reduction != "frame_mean":
            raise NotImplementedError("only reduction='frame_mean' (the reference Model's setting, vqvae.py:24)")
        self.register_buffer("emb_init", torch.tensor(0).bool())
        self.register_buffer("emb_sum", torch.zeros(z_num, z_dim))
        self.register_buffer("emb_elem", torch.ones(z_num))
        self.register_buffer("embeddings", torch.zeros(z_num, z_dim))
        self.mu, self.z_num, self.z_dim, self.threshold = mu, z_num, z_dim, threshold
        self.reduction = reduction
        self.quantize = True
        self.update = True
        self._init_host = None  # host mirror of emb_init (avoids a device sync per step)

    @property
    def initialized(self):
        if self._init_host is None:
            self._init_host = bool(self.emb_init.item())
        return self._init_host

    def mark_initialized(self):
        self.emb_init.fill_(True)
        self._init_host = True

    def _load_from_state_dict(self, *args, **kwargs):
        super()._load_from_state_dict(*args, **kwargs)
        self._init_host = None

    def encode(self, z, time_last=True):
        """Nearest-code indices of z (B, D, T) (layers_vq.py:236-252) on the HIP VQ kernel."""
        if time_last:
            B, D, T = z.shape
            zf = z.transpose(1, 2).reshape(-1, D).float().contiguous()
        else:
            B, T, D = z.shape
            zf = z.reshape(-1, D).float().contiguous()
        n = zf.shape[0]
        idx = torch.empty(n, dtype=torch.int64, device=z.device)
        ops.vq_forward(zf, self.embeddings.contiguous(), idx, None, None, None)
        return idx.view(B, T)

    def decode(self, z_id, time_last=True):
        """Codebook gather (layers_vq.py:255-265)."""
        B, T = z_id.shape
        out = torch.empty(B * T, self.z_dim, device=z_id.device)
        ops.gather_rows(self.embeddings.contiguous(), z_id.reshape(-1).contiguous(), out)
        out = out.view(B, T, -1)
        return out.transpose(1, 2).contiguous() if time_last else out

    def extra_repr(self):
        return f"{self.z_num}, {self.z_dim}, mu={self.mu}, threshold={self.threshold}"


class VectorQuantizer(nn.Module):
    """Straight-through codebook (layers_vq.py:9-163): the codebook is the
    parameter `embeddings` [K, D] (randn, normalised at construction when
    `normalize`, :13-20).  Training runs in the engine (vqx_vq_normalize /
    vqx_vq_forward / vqx_vq_plain_bwd); encode / decode here run the same HIP
    kernels without the in-place renormalisation, as the reference's do."""

    def __init__(self, z_num, z_dim, normalize=False, reduction="frame_mean"):
        super().__init__()
        if reduction != "frame_mean":
            raise NotImplementedError("only reduction='frame_mean' (the reference Model's setting, vqvae.py:31)")
        self.target_norm = 1.0 if normalize else None
        self.embeddings = nn.Parameter(torch.randn(z_num, z_dim, requires_grad=True))
        self.embed_norm()
        self.z_num, self.z_dim, self.normalize, self.reduction = z_num, z_dim, normalize, reduction
        self.quantize = True

    def embed_norm(self):
        """In-place row renormalisation of the codebook (layers_vq.py:28-33)."""
        if self.target_norm:
            with torch.no_grad():
                self.embeddings.mul_(self.target_norm / self.embeddings.norm(dim=1, keepdim=True))

    def _codebook(self):
        E = self.embeddings.detach().float().contiguous()
        if not self.normalize:
            return E
        K = E.shape[0]
        Ew = E.clone()
        emb = torch.empty_like(E)
        elen = torch.empty(K, device=E.device)
        zdummy = torch.zeros(1, E.shape[1], device=E.device)
        ops.vq_normalize(zdummy, Ew, torch.empty_like(zdummy), torch.empty(1, device=E.device), emb, elen,
                         torch.empty(2, device=E.device))
        # Ew was renormalised (not written back: encode/decode do not call embed_norm);
        # emb = Ew/||Ew|| == the reference's target_norm * E / ||E|| up to rounding
        return emb

    def encode(self, z, time_last=True):
        """Nearest-code indices (layers_vq.py:36-58) on the HIP VQ kernel."""
        if time_last:
            B, D, T = z.shape
            zf = z.transpose(1, 2).reshape(-1, D).float().contiguous()
        else:
            B, T, D = z.shape
            zf = z.reshape(-1, D).float().contiguous()
        n = zf.shape[0]
        emb = self._codebook()
        if self.normalize:
            zn, zl = torch.empty_like(zf), torch.empty(n, device=z.device)
            ops.vq_normalize(zf, emb.clone(), zn, zl, torch.empty_like(emb), torch.empty(emb.shape[0], device=z.device),
                             torch.empty(n // 4 + 2, device=z.device))
            zf = zn
        idx = torch.empty(n, dtype=torch.int64, device=z.device)
        ops.vq_forward(zf, emb, idx, None, None, None)
        return idx.view(B, T)

    def decode(self, z_id, time_last=True):
        """Codebook gather (layers_vq.py:61-76)."""
        B, T = z_id.shape
        out = torch.empty(B * T, self.z_dim, device=z_id.device)
        ops.gather_rows(self._codebook(), z_id.reshape(-1).contiguous(), out)
        out = out.view(B, T, -1)
        return out.transpose(1, 2).contiguous() if time_last else out

    def extra_repr(self):
        return f"{self.z_num}, {self.z_dim}" + (", normalize=True" if self.normalize else "")


class Jitter(nn.Module):
    """Jitter (layers_vq.py:337-383).  The neighbour map is drawn on the host
    numpy stream exactly as the reference does (so seeded runs match) and the
    time gather is a HIP kernel inside the engine.  Note the reference's
    indexing replaces a frame with probability 1-p (layers_vq.py:365)."""

    def __init__(self, probability=0.12):
        super().__init__()
        self.probability = probability

    def extra_repr(self):
        return f"jitter_prob={self.probability}"
