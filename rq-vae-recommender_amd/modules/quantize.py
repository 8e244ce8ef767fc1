"""One residual-quantization level — drop-in for reference modules/quantize.py.

Public surface kept from the reference (names, argument meaning, return types, state-dict keys
``embedding.weight`` / ``out_proj.*``, assertions and exceptions):
  QuantizeForwardMode (:16-20), QuantizeDistance (:23-25), QuantizeOutput (:28-31),
  efficient_rotation_trick_transform (:34-45), Quantize (:48-156).

Execution: the L2-distance path (every config) runs the fused HIP kernel
``rqvae_hip.ops.rq_quantize`` — MFMA fp32 distance + argmin + codeword gather + rotation trick /
STE / eval output + VQ loss in one launch, and the matching VJP with a deterministic codebook
gradient. GUMBEL_SOFTMAX training with the L2 distance (the reference's default codebook mode, differentiable
through the full distance matrix) and the COSINE distance run as GPU torch composites of the same math; the
Gumbel row kernels rq_gumbel_softmax_fwd / _bwd are parity-tested and opt-in (GUMBEL_HIP = True: slower than
the composite's library GEMMs as measured).
"""
from enum import Enum
from typing import NamedTuple

import torch
from torch import nn
from torch import Tensor
from torch.nn import functional as F

import distributions.gumbel as _gumbel
from distributions.gumbel import gumbel_softmax_sample
from init.kmeans import kmeans_init_
from modules.loss import QuantizeLoss
from modules.normalize import L2NormalizationLayer
from rqvae_hip import ops as hip_ops

from modules.ginlite import gin as _gin   # gin-config, or the built-in subset when gin is absent


# GUMBEL_HIP = True: the training-mode Gumbel-softmax quantize on rq_gumbel_softmax_fwd / _bwd (parity-tested);
# default: the GPU torch composite — measured faster (ML-32M level shape fwd+bwd 1.31 vs 2.35 ms: the row
# kernels' per-lane K x D dot loops lose to the library GEMMs). Tests set the attribute.
GUMBEL_HIP = False


class QuantizeForwardMode(Enum):
    GUMBEL_SOFTMAX = 1
    STE = 2
    ROTATION_TRICK = 3


class QuantizeDistance(Enum):
    L2 = 1
    COSINE = 2


_gin.constants_from_enum(QuantizeForwardMode, module="modules.quantize")


class QuantizeOutput(NamedTuple):
    embeddings: Tensor
    ids: Tensor
    loss: Tensor


def efficient_rotation_trick_transform(u, q, e):
    """Rotation trick (arXiv 2410.06424 §4.2): e - 2 (e.w) w + 2 (e.u) q with w = normalize(u+q)
    detached and u, q detached; (B, D) rows. Same contract as the reference helper (:34-45);
    the fused kernel evaluates exactly this expression per row."""
    w = F.normalize(u + q, p=2, dim=1, eps=1e-6).detach()
    ew = (e * w).sum(-1, keepdim=True)
    eu = (e * u.detach()).sum(-1, keepdim=True)
    return (e - 2 * (ew * w) + 2 * (eu * q.detach())).squeeze()


def fused_mode(forward_mode: QuantizeForwardMode, training: bool):
    """Kernel mode for a (mode, training) pair, or None when no fused kernel applies."""
    if not training:
        return hip_ops.MODE_EVAL
    if forward_mode == QuantizeForwardMode.ROTATION_TRICK:
        return hip_ops.MODE_ROTATION
    if forward_mode == QuantizeForwardMode.STE:
        return hip_ops.MODE_STE
    return None


class Quantize(nn.Module):
    def __init__(
        self,
        embed_dim: int,
        n_embed: int,
        do_kmeans_init: bool = True,
        codebook_normalize: bool = False,
        sim_vq: bool = False,
        commitment_weight: float = 0.25,
        forward_mode: QuantizeForwardMode = QuantizeForwardMode.GUMBEL_SOFTMAX,
        distance_mode: QuantizeDistance = QuantizeDistance.L2,
    ) -> None:
        super().__init__()
        self.embed_dim = embed_dim
        self.n_embed = n_embed
        self.embedding = nn.Embedding(n_embed, embed_dim)
        self.forward_mode = forward_mode
        self.distance_mode = distance_mode
        self.do_kmeans_init = do_kmeans_init
        self.kmeans_initted = False
        self.commitment_weight = commitment_weight
        proj = nn.Linear(embed_dim, embed_dim, bias=False) if sim_vq else nn.Identity()
        norm = L2NormalizationLayer(dim=-1) if codebook_normalize else nn.Identity()
        self.out_proj = nn.Sequential(proj, norm)
        self.quantize_loss = QuantizeLoss(commitment_weight)
        nn.init.uniform_(self.embedding.weight)   # reference _init_weights (:86-89)

    @property
    def weight(self) -> Tensor:
        return self.embedding.weight

    @property
    def device(self) -> torch.device:
        return self.embedding.weight.device

    def _init_weights(self) -> None:
        for m in self.modules():
            if isinstance(m, nn.Embedding):
                nn.init.uniform_(m.weight)

    @torch.no_grad()
    def _kmeans_init(self, x) -> None:
        kmeans_init_(self.embedding.weight, x=x)
        self.kmeans_initted = True

    def get_item_embeddings(self, item_ids) -> Tensor:
        return self.out_proj(self.embedding(item_ids))

    def codebook(self) -> Tensor:
        return self.out_proj(self.embedding.weight)

    def needs_init(self) -> bool:
        return self.do_kmeans_init and not self.kmeans_initted

    def forward(self, x, temperature) -> QuantizeOutput:
        assert x.shape[-1] == self.embed_dim
        if self.needs_init():
            self._kmeans_init(x=x)
        codebook = self.codebook()
        if self.distance_mode == QuantizeDistance.L2:
            mode = fused_mode(self.forward_mode, self.training)
            if mode is not None:
                emb, _, ids, qloss, _ = hip_ops.rq_quantize(x, codebook.unsqueeze(0), mode, self.commitment_weight)
                return QuantizeOutput(embeddings=emb[0], ids=ids[:, 0], loss=qloss)
            if (self.training and self.forward_mode == QuantizeForwardMode.GUMBEL_SOFTMAX and GUMBEL_HIP
                    and hip_ops.gumbel_softmax_supported(x, codebook)):
                # the noise is drawn exactly as the reference's gumbel_softmax_sample draws it (torch.rand)
                noise = _gumbel.sample_gumbel((x.shape[0], codebook.shape[0]), x.device)
                emb, ids = hip_ops.gumbel_softmax_quantize(x, codebook, noise, temperature)
                return QuantizeOutput(embeddings=emb, ids=ids, loss=self.quantize_loss(query=x, value=emb))
        elif self.distance_mode != QuantizeDistance.COSINE:
            raise Exception("Unsupported Quantize distance mode.")
        return self._composite_forward(x, codebook, temperature)

    def _composite_forward(self, x, codebook, temperature) -> QuantizeOutput:
        """GUMBEL_SOFTMAX and COSINE (no config uses them): the reference math as GPU torch ops."""
        hip_ops.require_gpu(x, what="Quantize")
        if self.distance_mode == QuantizeDistance.L2:
            dist = (x ** 2).sum(axis=1, keepdim=True) + (codebook.T ** 2).sum(axis=0, keepdim=True) - 2 * x @ codebook.T
        else:
            dist = -((x / x.norm(dim=1, keepdim=True)) @ codebook.T / codebook.T.norm(dim=0, keepdim=True))
        ids = dist.detach().argmin(dim=1)
        if not self.training:
            emb_out = self.get_item_embeddings(ids)
            return QuantizeOutput(embeddings=emb_out, ids=ids, loss=self.quantize_loss(query=x, value=emb_out))
        if self.forward_mode == QuantizeForwardMode.GUMBEL_SOFTMAX:
            emb = gumbel_softmax_sample(-dist, temperature=temperature, device=self.device) @ codebook
            emb_out = emb
        elif self.forward_mode == QuantizeForwardMode.STE:
            emb = self.get_item_embeddings(ids)
            emb_out = x + (emb - x).detach()
        elif self.forward_mode == QuantizeForwardMode.ROTATION_TRICK:
            emb = self.get_item_embeddings(ids)
            xn = x.norm(dim=-1, keepdim=True)
            en = emb.norm(dim=-1, keepdim=True)
            emb_out = efficient_rotation_trick_transform(x / (xn + 1e-8), emb / (en + 1e-8), x)
            emb_out = emb_out * (en / (xn + 1e-6)).detach()
        else:
            raise Exception("Unsupported Quantize forward mode.")
        return QuantizeOutput(embeddings=emb_out, ids=ids, loss=self.quantize_loss(query=x, value=emb))
