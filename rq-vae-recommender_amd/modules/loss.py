"""Per-sample losses — reference semantics: modules/loss.py:5-42.

On the fused hot path the VQ loss is produced inside the rq_quantize kernels; these modules
serve the generic per-level path and the reconstruction term.
"""
import torch.nn.functional as F
from torch import nn

__all__ = ["ReconstructionLoss", "CategoricalReconstuctionLoss", "QuantizeLoss"]


def _sq_err(a, b):
    d = a - b
    return (d * d).sum(dim=-1)


class ReconstructionLoss(nn.Module):
    """Row-wise sum of squared errors."""

    def forward(self, x_hat, x):
        return _sq_err(x_hat, x)


class CategoricalReconstuctionLoss(nn.Module):
    """Squared error on the dense head plus summed BCE-with-logits on the last n_cat_feats
    columns (the reference's class name, typo included, is the API)."""

    def __init__(self, n_cat_feats: int) -> None:
        super().__init__()
        self.n_cat_feats = n_cat_feats
        self.reconstruction_loss = ReconstructionLoss()

    def forward(self, x_hat, x):
        n = self.n_cat_feats
        dense = self.reconstruction_loss(x_hat[:, :-n], x[:, :-n])
        if n <= 0:
            return dense
        bce = F.binary_cross_entropy_with_logits(x_hat[:, -n:], x[:, -n:], reduction="none")
        return dense + bce.sum(dim=-1)


class QuantizeLoss(nn.Module):
    """codebook term |sg(query) - value|^2 + commitment_weight * |query - sg(value)|^2."""

    def __init__(self, commitment_weight: float = 1.0) -> None:
        super().__init__()
        self.commitment_weight = commitment_weight

    def forward(self, query, value):
        codebook_term = _sq_err(query.detach(), value)
        commit_term = _sq_err(query, value.detach())
        return codebook_term + self.commitment_weight * commit_term
