"""RQ-VAE — drop-in for reference modules/rqvae.py (RqVaeOutput :22-26, RqVaeComputedLosses
:29-34, RqVae :37-165; same constructor, methods, outputs and state-dict keys
``encoder.mlp.*``, ``decoder.mlp.*``, ``layers.{l}.embedding.weight``).

Hot path: ``get_semantic_ids`` runs all L levels in ONE fused HIP launch
(rqvae_hip.ops.rq_quantize: MFMA fp32 cdist -> argmin -> rotation trick / STE / eval -> VQ loss
-> residual update, chained on-chip) and its VJP with a deterministic codebook gradient.
``p_unique_ids`` uses a hash-count kernel (O(B L)) instead of the reference's O(B^2 L) mask.
The reference wraps forward in torch.compile(mode="reduce-overhead"); this build instead
exposes a whole-step hipGraph capture (rqvae_hip.graph) and never invokes inductor.
"""
from typing import List, NamedTuple

import torch
from torch import nn
from torch import Tensor

from data.schemas import SeqBatch
from modules.encoder import MLP
from modules.loss import CategoricalReconstuctionLoss, ReconstructionLoss
from modules.normalize import L2NormalizationLayer, l2norm
from modules.quantize import Quantize, QuantizeDistance, QuantizeForwardMode, fused_mode
from rqvae_hip import ops as hip_ops

# As the reference (modules/rqvae.py:19): fp32 matmuls at 'high' precision. On gfx950 (no xf32)
# the MLP matmuls then run split-bf16 (rqvae_hip.ops.gemm_bf16x3); 'highest' restores exact fp32.
torch.set_float32_matmul_precision('high')


class RqVaeOutput(NamedTuple):
    embeddings: Tensor      # (B, D, L)
    residuals: Tensor       # (B, D, L)
    sem_ids: Tensor         # (B, L) int64
    quantize_loss: Tensor   # (B,)


class RqVaeComputedLosses(NamedTuple):
    loss: Tensor
    reconstruction_loss: Tensor
    rqvae_loss: Tensor
    embs_norm: Tensor       # (B, L)
    p_unique_ids: Tensor    # 0-d float


class RqVae(nn.Module):
    def __init__(
        self,
        input_dim: int,
        embed_dim: int,
        hidden_dims: List[int],
        codebook_size: int,
        codebook_kmeans_init: bool = True,
        codebook_normalize: bool = False,
        codebook_sim_vq: bool = False,
        codebook_mode: QuantizeForwardMode = QuantizeForwardMode.GUMBEL_SOFTMAX,
        n_layers: int = 3,
        commitment_weight: float = 0.25,
        n_cat_features: int = 18,
    ) -> None:
        # plain kwargs (the reference pickles `self` via locals(); SURVEY A-13)
        self._config = dict(input_dim=input_dim, embed_dim=embed_dim, hidden_dims=list(hidden_dims),
                            codebook_size=codebook_size, codebook_kmeans_init=codebook_kmeans_init,
                            codebook_normalize=codebook_normalize, codebook_sim_vq=codebook_sim_vq,
                            codebook_mode=codebook_mode, n_layers=n_layers, commitment_weight=commitment_weight,
                            n_cat_features=n_cat_features)
        super().__init__()
        self.input_dim = input_dim
        self.embed_dim = embed_dim
        self.hidden_dims = hidden_dims
        self.n_layers = n_layers
        self.codebook_size = codebook_size
        self.commitment_weight = commitment_weight
        self.n_cat_feats = n_cat_features
        self.layers = nn.ModuleList([
            Quantize(embed_dim=embed_dim, n_embed=codebook_size, forward_mode=codebook_mode,
                     do_kmeans_init=codebook_kmeans_init, codebook_normalize=(i == 0 and codebook_normalize),
                     sim_vq=codebook_sim_vq, commitment_weight=commitment_weight)
            for i in range(n_layers)
        ])
        self.encoder = MLP(input_dim=input_dim, hidden_dims=hidden_dims, out_dim=embed_dim,
                           normalize=codebook_normalize)
        self.decoder = MLP(input_dim=embed_dim, hidden_dims=list(hidden_dims)[::-1], out_dim=input_dim,
                           normalize=True)
        self.reconstruction_loss = (CategoricalReconstuctionLoss(n_cat_features) if n_cat_features != 0
                                    else ReconstructionLoss())

    @property
    def config(self) -> dict:
        return self._config

    @property
    def device(self) -> torch.device:
        return next(self.encoder.parameters()).device

    def load_pretrained(self, path: str) -> None:
        """Load a checkpoint {"iter", "model", ...}. Only tensor payloads are accepted
        (weights_only=True): reference checkpoints that pickle the module object itself must be
        re-saved as a plain state dict first."""
        state = torch.load(path, map_location=self.device, weights_only=True)
        self.load_state_dict(state["model"])
        print(f"---Loaded RQVAE Iter {state['iter']}---")

    def encode(self, x: Tensor) -> Tensor:
        return self.encoder(x)

    def decode(self, x: Tensor) -> Tensor:
        return self.decoder(x)

    # ----------------------------------------------------------------- semantic ids
    def _fused_kernel_mode(self):
        modes = {fused_mode(layer.forward_mode, self.training) for layer in self.layers}
        if len(modes) != 1 or None in modes:
            return None
        if any(layer.distance_mode != QuantizeDistance.L2 or layer.needs_init() for layer in self.layers):
            return None
        return modes.pop()

    def quantize_levels(self, res0: Tensor, gumbel_t: float, with_norms: bool = False):
        """All levels -> (emb (L,B,D), res (L,B,D), ids (B,L), qloss (B,), emb_sum (B,D)
        [, |emb| (L,B) without grad when with_norms])."""
        mode = self._fused_kernel_mode()
        if mode is not None:
            if all(isinstance(m, nn.Identity) for layer in self.layers for m in layer.out_proj):   # codebook() == weight
                codebooks = hip_ops.stack_params([layer.embedding.weight for layer in self.layers])
            else:
                codebooks = torch.stack([layer.codebook() for layer in self.layers])
            return hip_ops.rq_quantize(res0, codebooks, mode, self.commitment_weight, with_norms)
        # generic per-level path (k-means init pending, gumbel / cosine layers)
        res, qloss = res0, 0
        embs, ress, ids = [], [], []
        for layer in self.layers:
            ress.append(res)
            q = layer(res, temperature=gumbel_t)
            qloss = qloss + q.loss
            res = res - q.embeddings
            embs.append(q.embeddings)
            ids.append(q.ids)
        emb = torch.stack(embs)
        out = (emb, torch.stack(ress), torch.stack(ids, 1), qloss, emb.sum(0))
        if with_norms:
            with torch.no_grad():
                out += (hip_ops.row_norms(emb),)     # emb.norm(dim=-1) over (L, B, D)
        return out

    def get_semantic_ids(self, x: Tensor, gumbel_t: float = 0.001) -> RqVaeOutput:
        emb, res, ids, qloss, _ = self.quantize_levels(self.encode(x), gumbel_t)
        return RqVaeOutput(embeddings=emb.permute(1, 2, 0), residuals=res.permute(1, 2, 0), sem_ids=ids,
                           quantize_loss=qloss)

    def forward(self, batch: SeqBatch, gumbel_t: float) -> RqVaeComputedLosses:
        # every encoder / decoder GEMM weight split once for the step, in one launch (the fused chains take
        # their planes from the scope; two chains split separately were two launches)
        weights = [m.weight for mlp in (self.encoder.mlp, self.decoder.mlp) for m in mlp if isinstance(m, nn.Linear)]
        with hip_ops.weight_split_scope(weights):
            return self._forward(batch, gumbel_t)

    def _forward(self, batch: SeqBatch, gumbel_t: float) -> RqVaeComputedLosses:
        x = batch.x
        # the level loop also returns embs_norm = |emb_l| (modules/rqvae.py:151 of the reference),
        # written from the fused kernel's level epilogue
        emb, _, ids, qloss, emb_sum, emb_norms = self.quantize_levels(self.encode(x), gumbel_t, with_norms=True)
        n = self.n_cat_feats
        head = self.decoder.mlp
        if n == 0 and isinstance(head[-1], L2NormalizationLayer) and x.dtype == torch.float32:
            fused = self.decoder._fused_chain(emb_sum)
            if fused is not None and x.shape[-1] % 4 == 0:
                # 'high': the decoder MLP chain + l2norm + ReconstructionLoss as one node whose
                # backward hands the split output gradient straight to the chain's GEMMs
                reconstruction = hip_ops.mlp_l2norm_recon(emb_sum, x, fused[0], fused[1])
            else:
                # decoder's final l2norm + ReconstructionLoss fused into one HIP row kernel (fwd + bwd)
                reconstruction = hip_ops.l2norm_recon_loss(self.decoder.body(emb_sum), x)
        else:
            x_hat = self.decode(emb_sum)
            if n > 0:   # the reference's cat is a no-op for n == 0 (SURVEY A-10)
                x_hat = torch.cat([l2norm(x_hat[..., :-n]), x_hat[..., -n:]], axis=-1)
            reconstruction = self.reconstruction_loss(x_hat, x)
        # loss = mean(recon + qloss) and the two logged means in one deterministic pass
        loss, recon_mean, rq_mean = hip_ops.loss_means(reconstruction, qloss)
        with torch.no_grad():
            embs_norm = emb_norms.T
            p_unique_ids = hip_ops.unique_fraction(ids, self.codebook_size)
        return RqVaeComputedLosses(loss=loss, reconstruction_loss=recon_mean, rqvae_loss=rq_mean,
                                   embs_norm=embs_norm, p_unique_ids=p_unique_ids)
