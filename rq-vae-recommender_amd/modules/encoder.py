"""Bias-free MLP — reference semantics: modules/encoder.py:7-36.

Layer order inside ``self.mlp`` (and therefore the state-dict keys ``mlp.{i}.weight``) is the
reference's: Linear, SiLU, [Dropout], ..., Linear, then L2 norm or Identity. Forward and data-grad
GEMMs run on hipBLASLt through torch; weight gradients on the split-K HIP kernel
(modules.linear.Linear); the RQ hot path around them is HIP (rqvae_hip.ops).
"""
from typing import List

from torch import nn

from modules.linear import Linear
from rqvae_hip import ops as hip_ops
from modules.normalize import L2NormalizationLayer


def _layer_stack(dims, dropout, normalize):
    seq = nn.Sequential()
    last = len(dims) - 2
    for i in range(last + 1):
        seq.append(Linear(dims[i], dims[i + 1], bias=False))
        if i < last:
            seq.append(nn.SiLU())
            if dropout:
                seq.append(nn.Dropout(dropout))
    seq.append(L2NormalizationLayer() if normalize else nn.Identity())
    return seq


class MLP(nn.Module):
    def __init__(self, input_dim: int, hidden_dims: List[int], out_dim: int, dropout: float = 0.0,
                 normalize: bool = False) -> None:
        super().__init__()
        self.input_dim, self.hidden_dims, self.out_dim, self.dropout = input_dim, hidden_dims, out_dim, dropout
        self.mlp = _layer_stack([input_dim, *hidden_dims, out_dim], dropout, normalize)

    def forward(self, x):
        assert x.shape[-1] == self.input_dim, f"Invalid input dim: Expected {self.input_dim}, found {x.shape[-1]}"
        mods = self.mlp
        i, n = 0, len(mods)
        while i < n:
            m = mods[i]
            nxt = mods[i + 1] if i + 1 < n else None
            if (isinstance(m, nn.SiLU) and isinstance(nxt, nn.Dropout) and nxt.training and nxt.p > 0
                    and hip_ops.dropout_fusable(x)):
                x = hip_ops.silu_dropout(x, nxt.p)   # SiLU + Dropout in one HIP pass
                i += 2
                continue
            x = m(x)
            i += 1
        return x
