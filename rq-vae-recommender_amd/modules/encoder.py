"""Bias-free MLP — reference semantics: modules/encoder.py:7-36.

Layer order inside ``self.mlp`` (and therefore the state-dict keys ``mlp.{i}.weight``) is the
reference's: Linear, SiLU, [Dropout], ..., Linear, then L2 norm or Identity. At matmul precision
'high' (the reference's import-time setting) the whole chain is one fused node
(rqvae_hip.ops.MLPFunction: split-bf16 GEMMs with SiLU / dropout in their epilogues); at
'highest' each Linear runs exact fp32 (modules.linear.Linear).
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

    def _fused_chain(self, x):
        """(weights, p) when the Linear-SiLU-[Dropout] chain can run as one fused 'high'-precision
        node (rqvae_hip.ops.MLPFunction), else None."""
        if not hip_ops.matmul_high():
            return None
        weights, p = [], 0.0
        for m in self.mlp:
            if isinstance(m, Linear):
                if m.bias is not None:
                    return None
                weights.append(m.weight)
            elif isinstance(m, nn.Dropout):
                p = m.p if m.training else 0.0
        return (weights, p) if hip_ops.mlp_fusable(x, weights) else None

    def body(self, x):
        """The Linear / SiLU / [Dropout] chain without the final L2 norm / Identity."""
        fused = self._fused_chain(x)
        if fused is not None:
            return hip_ops.mlp_chain(x, fused[0], fused[1])
        mods = self.mlp
        i, n = 0, len(mods) - 1
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

    def forward(self, x):
        assert x.shape[-1] == self.input_dim, f"Invalid input dim: Expected {self.input_dim}, found {x.shape[-1]}"
        return self.mlp[-1](self.body(x))   # then L2 norm / Identity
