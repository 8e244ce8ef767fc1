"""Jagged multi-head attention — drop-in for reference modules/transformer/attention.py.

Kept: ``AttentionInput``, ``Attend(d_out, num_heads, head_dim, dropout)`` with
``jagged_forward(qu, ke, va, is_causal)`` (:113-124) and ``MultiHeadAttention(d_in, d_out,
num_heads, cross_attn=False, dropout=0.0, qkv_bias=False, enable_kv_cache=False)`` with
``forward(x, x_kv=None, padding_mask=None, is_causal=True, jagged=False, use_cache=False)``
(:147-233), module names ``qkv`` / ``q`` / ``kv`` / ``proj`` and the reference's assertions
and exceptions (KV cache unsupported :161; dense attention raises :228-229).

MI355X path: NJT q/k/v values (row-strided views of the fused projection output, consumed in
place) go to the HIP varlen attention kernels (rqvae_hip.ops.varlen_attention: fp32 / split-bf16
MFMA, online softmax, a one-pass fused backward per shape class — long key ranges, short
self-attention, few-query cross-attention — with deterministic, fixed-order dQ sums; the two-pass
form stays as an A/B policy). Attention dropout is always 0, as in the reference (Attend is built
with dropout=False).
"""
from typing import Optional, Union

import torch
from torch import nn
from torch import Tensor

from ops.jagged import Jagged, as_jagged
from rqvae_hip import ops as hip_ops
from modules.linear import Linear

AttentionInput = Union[Tensor, "torch.nested.Tensor", Jagged]


def _wrap_like(values: Tensor, like):
    """NJT over `values` sharing `like`'s offsets (hence its ragged dimension)."""
    kw = {}
    for name, key in (("_maybe_min_seqlen", "min_seqlen"), ("_maybe_max_seqlen", "max_seqlen")):
        v = getattr(like, name, None)
        if v is not None:
            kw[key] = int(v)
    return torch.nested.nested_tensor_from_jagged(values, like.offsets(), **kw)


class Attend(nn.Module):
    def __init__(self, d_out, num_heads, head_dim, dropout):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = head_dim
        self.d_out = d_out
        self.dropout = dropout

    def jagged_forward(self, qu, ke, va, is_causal: bool):
        """softmax(q k^T / sqrt(head_dim)) v per sequence; NJT (B, j, H*hd) in and out (a dense
        ``Jagged`` in gives a ``Jagged`` out)."""
        assert not (self.training and self.dropout), "attention dropout is not supported (reference forces 0)"
        jq, jk, jv = as_jagged(qu), as_jagged(ke), as_jagged(va)
        out = hip_ops.varlen_attention(jq.values(), jk.values(), jv.values(), jq.offsets(), jk.offsets(),
                                       self.num_heads, bool(is_causal), jq.max_len, jk.max_len)
        return jq.with_values(out) if isinstance(qu, Jagged) else _wrap_like(out, qu)

    def forward(self, qkv: Tensor, is_causal: bool = False) -> Tensor:
        raise Exception("Unjagged attention currently not supported.")


class MultiHeadAttention(nn.Module):
    def __init__(self, d_in, d_out, num_heads, cross_attn=False, dropout=0.0, qkv_bias=False,
                 enable_kv_cache=False) -> None:
        super().__init__()
        assert d_out % num_heads == 0, "embed_dim is indivisible by num_heads"
        assert not enable_kv_cache, "KV Cache currently not supported"
        self.cross_attn = cross_attn
        self.num_heads = num_heads
        self.head_dim = d_out // num_heads
        self.d_out = d_out
        self.enable_kv_cache = enable_kv_cache
        if cross_attn:
            self.q = Linear(d_in, d_out, bias=qkv_bias)
            self.kv = Linear(d_in, 2 * d_out, bias=qkv_bias)
        else:
            self.qkv = Linear(d_in, 3 * d_out, bias=qkv_bias)
        self.proj = Linear(d_out, d_out, bias=False)
        self.attend = Attend(self.d_out, self.num_heads, self.head_dim, dropout=False)
        self._kv_cache = None

    @property
    def kv_cache(self):
        return self._kv_cache

    def forward(self, x: AttentionInput, x_kv: Optional[AttentionInput] = None, padding_mask: Optional[Tensor] = None,
                is_causal: Optional[bool] = True, jagged: bool = False, use_cache: bool = False,
                residual: Optional[Tensor] = None, kv_values: Optional[Tensor] = None,
                proj_values: Optional[Tensor] = None) -> AttentionInput:
        """`residual` (this build's extension, default None = the reference's contract): values
        (T, d_out) added to the output projection inside its GEMM (out = proj(ctx) + residual).
        `kv_values` (extension, cross-attention): this layer's `self.kv(x_kv)` already computed by the
        decoder's hoisted projection of the shared context (TransformerDecoder.forward).
        `proj_values` (extension): `self.qkv(x)` (self-attention) or `self.q(x)` (cross-attention) already
        computed — by the block's paired projection launch (TransformerBlock._forward_fork)."""
        assert not self.cross_attn or x_kv is not None, "Found null x_kv in cross attn. layer"
        if not jagged:
            raise Exception("Unjagged attention currently not supported.")
        jx = as_jagged(x)
        # q/k/v stay column blocks of the packed projection outputs (read in place through row
        # strides); the backward writes their gradients into one buffer per projection (no cat)
        if self.cross_attn:
            jkv = as_jagged(x_kv)
            kv = self.kv(jkv.values()) if kv_values is None else kv_values
            q = self.q(jx.values()) if proj_values is None else proj_values
            ctx = hip_ops.varlen_attention_packed(q, kv, jx.offsets(),
                                                  jkv.offsets(), self.num_heads, bool(is_causal), jx.max_len,
                                                  jkv.max_len)
        else:
            qkv = self.qkv(jx.values()) if proj_values is None else proj_values
            ctx = hip_ops.varlen_attention_packed(qkv, None, jx.offsets(), jx.offsets(),
                                                  self.num_heads, bool(is_causal), jx.max_len, jx.max_len)
        out = self.proj(ctx) if residual is None else hip_ops.linear_add(ctx, self.proj.weight, residual)
        return jx.with_values(out) if isinstance(x, Jagged) else _wrap_like(out, x)
