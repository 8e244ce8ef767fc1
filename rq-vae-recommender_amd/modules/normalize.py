"""Normalisation layers — reference semantics: modules/normalize.py:7-32.

* ``l2norm``: divide by max(||x||_2, eps) along ``dim`` (eps 1e-12), i.e. F.normalize.
* ``RMSNorm``: y = w * x / sqrt(mean(x^2, -1) + eps), evaluated in fp32 and cast back to the
  input dtype before the weight multiply. Dense fp32 device tensors run the fused HIP kernels
  (rqvae_hip.ops.rmsnorm: one HBM pass each way); jagged NJTs and CPU tensors take torch's ops
  (it only touches the last, dense axis).
"""
import torch
from torch import nn
from torch.nn import functional as F

from rqvae_hip import ops as hip_ops

__all__ = ["l2norm", "L2NormalizationLayer", "RMSNorm"]


def l2norm(x, dim=-1, eps=1e-12):
    return F.normalize(x, p=2, dim=dim, eps=eps)


class L2NormalizationLayer(nn.Module):
    def __init__(self, dim=-1, eps=1e-12) -> None:
        super().__init__()
        self.dim, self.eps = dim, eps

    def forward(self, x):
        return l2norm(x, self.dim, self.eps)


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float = 1e-6) -> None:
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))

    def _norm(self, x):
        inv_rms = torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + self.eps)
        return x * inv_rms

    def forward(self, x):
        if hip_ops.rmsnorm_supported(x, self.weight):
            return hip_ops.rmsnorm(x, self.weight, self.eps)
        y = self._norm(x.float()).type_as(x)
        return y * self.weight

    def forward_dropout(self, x, dropout: nn.Dropout):
        """dropout(self(x)) — one fused HIP pass (mask regenerated in backward) when training on the
        device; the two separate ops otherwise."""
        if dropout.training and dropout.p > 0 and hip_ops.rmsnorm_supported(x, self.weight):
            return hip_ops.rmsnorm(x, self.weight, self.eps, dropout.p)
        return dropout(self(x))
