"""Pre-norm transformer encoder/decoder over jagged sequences — drop-in for reference
modules/transformer/model.py (TransformerBlock :21-92, TransformerDecoder :95-136,
TransformerEncoderDecoder :139-188; same constructor arguments, submodule names and so
state-dict keys).

Block semantics reproduced exactly (SURVEY A-11):
  h   = x + SelfAttn(Dropout(attn_norm(x)))
  h  += CrossAttn(Dropout(cross_attn_norm(x)), context)      # norm of x, not h
  out = h + Dropout(MLP(RMSNorm(h)))                          # `ffn_norm` exists but is unused
The encoder output is cached in eval mode (`cached_enc_output`) exactly like the reference.

Jagged inputs may be torch NJTs (drop-in) or dense ``ops.jagged.Jagged`` views; NJTs are
unwrapped once at the module boundary and every row-wise op (RMSNorm, dropout, Linear, residual
adds) runs on the dense (T, C) values, avoiding NJT's per-op Python dispatch.
"""
from typing import List, Optional

import torch
from torch import nn
from torch import Tensor

from modules.encoder import MLP
from modules.normalize import RMSNorm
from modules.transformer.attention import AttentionInput, MultiHeadAttention, _wrap_like
from ops.jagged import Jagged, as_jagged
from rqvae_hip import ops as hip_ops

# False selects the unfused form (tests / A-B probes set these module attributes):
_FF_RESIDUAL = True   # False: the feed-forward output as MLP + dropout_add
_HOIST_KV = True      # False: per-layer cross-attention K/V projections
_PAIR_PROJ = True     # False: the self-attention qkv and cross-attention q projections as two launches


class KVCacheOpsMixin:
    def reset_kv_cache(self) -> None:
        for layer in self.layers:
            layer.reset_kv_cache()

    def apply_to_kv_cache(self, fn) -> None:
        for layer in self.layers:
            layer.apply_to_kv_cache(fn)


class TransformerBlock(nn.Module):
    def __init__(self, d_in: int, d_out: int, dropout: float, num_heads: int, qkv_bias: bool,
                 mlp_hidden_dims: List[int] = [1024], do_cross_attn: bool = False,
                 enable_kv_cache: bool = True) -> None:
        super().__init__()
        self.d_in, self.d_out, self.num_heads = d_in, d_out, num_heads
        self.qkv_bias, self.do_cross_attn, self.enable_kv_cache = qkv_bias, do_cross_attn, enable_kv_cache
        self.attention = MultiHeadAttention(d_in=d_in, d_out=d_out, num_heads=num_heads, cross_attn=False,
                                            dropout=dropout, qkv_bias=qkv_bias, enable_kv_cache=enable_kv_cache)
        self.ff = nn.Sequential(
            RMSNorm(d_out),
            MLP(input_dim=d_out, hidden_dims=mlp_hidden_dims, out_dim=d_out, dropout=dropout, normalize=False),
            nn.Dropout(dropout),
        )
        self.attn_norm = RMSNorm(d_out)
        self.ffn_norm = RMSNorm(d_out)
        self.do = nn.Dropout(dropout)
        if do_cross_attn:
            self.cross_attention = MultiHeadAttention(d_in=d_out, d_out=d_out, num_heads=num_heads, cross_attn=True,
                                                      dropout=dropout, qkv_bias=qkv_bias)
            self.cross_attn_norm = RMSNorm(d_out)

    def forward(self, x: AttentionInput, x_kv: Optional[Tensor] = None, padding_mask: Optional[Tensor] = None,
                is_causal: Optional[bool] = True, jagged: Optional[bool] = False) -> AttentionInput:
        if not jagged:
            raise Exception("Unjagged attention currently not supported.")
        jx = as_jagged(x)
        jkv = as_jagged(x_kv) if x_kv is not None else None
        out = self._forward_jagged(jx, jkv, is_causal)
        return out if isinstance(x, Jagged) else _wrap_like(out.values(), x)

    def _fork_ok(self, xv) -> bool:
        norms = [self.attn_norm] + ([self.cross_attn_norm] if self.do_cross_attn else []) + [self.ff[0]]
        return (all(hip_ops.rmsnorm_supported(xv, n.weight) for n in norms) and
                len({n.eps for n in norms}) == 1)

    def _forward_jagged(self, jx: Jagged, jkv: Optional[Jagged], is_causal: bool, kv=None) -> Jagged:
        use_cache = not self.training and self.enable_kv_cache
        xv = jx.values()
        if self._fork_ok(xv):
            return self._forward_fork(jx, jkv, is_causal, use_cache, kv)
        # residual adds ride in the output-projection GEMMs' epilogue (h = x + MHA(..), h += CrossMHA(..))
        h = self.attention(jx.with_values(self.attn_norm.forward_dropout(xv, self.do)), is_causal=is_causal,
                           jagged=True, use_cache=use_cache, residual=xv).values()
        if self.do_cross_attn:
            h = self.cross_attention(x=jx.with_values(self.cross_attn_norm.forward_dropout(xv, self.do)), x_kv=jkv,
                                     is_causal=False, jagged=True, use_cache=use_cache, residual=h,
                                     kv_values=kv).values()
        norm, mlp, drop = self.ff
        n3 = norm(h)
        fused = self._ff_residual(mlp, drop, n3, h)
        if fused is not None:
            return jx.with_values(fused)
        y = mlp(n3)
        if drop.training and drop.p > 0 and hip_ops.dropout_fusable(h) and hip_ops.dropout_fusable(y):
            return jx.with_values(hip_ops.dropout_add(h, y, drop.p))   # h + Dropout(ff) in one pass
        return jx.with_values(h + drop(y))

    @staticmethod
    def _ff_residual(mlp, drop, x, h):
        """h + Dropout(MLP(x)) with the residual and the output dropout in the MLP chain's last GEMM
        epilogue (training with dropout at 'high' precision), else None."""
        if not (_FF_RESIDUAL and drop.training and drop.p > 0 and hasattr(mlp, "_fused_chain")
                and hip_ops.dropout_fusable(h)):
            return None
        chain = mlp._fused_chain(x)
        if chain is None or h.shape[-1] != chain[0][-1].shape[0] or h.dtype != torch.float32:
            return None
        return hip_ops.mlp_chain_residual(x, chain[0], chain[1], h, drop.p)

    def _forward_fork(self, jx: Jagged, jkv: Optional[Jagged], is_causal: bool, use_cache: bool,
                      kv=None) -> Jagged:
        """Same block, with x's fan-out (norm branches + residual) and h's (ff norm + residual) as
        hip_ops.rmsnorm_fork nodes: the residual gradients are added inside the norm backward kernels."""
        xv = jx.values()
        p = self.do.p if self.do.training else 0.0
        norm, mlp, drop = self.ff
        if self.do_cross_attn:
            n1, n2, xr = hip_ops.rmsnorm_fork(xv, self.attn_norm.eps, self.attn_norm.weight, p,
                                              self.cross_attn_norm.weight, p)
        else:
            n1, xr = hip_ops.rmsnorm_fork(xv, self.attn_norm.eps, self.attn_norm.weight, p)
        qkv = q2 = None
        if self.do_cross_attn and _PAIR_PROJ and self._pair_ok(n1, n2):
            # the two projections of x's two norms are independent: one paired launch
            qkv, q2 = hip_ops.linear_pair(n1, self.attention.qkv.weight, n2, self.cross_attention.q.weight)
        h = self.attention(jx.with_values(n1), is_causal=is_causal, jagged=True, use_cache=use_cache,
                           residual=xr, proj_values=qkv).values()
        if self.do_cross_attn:
            h = self.cross_attention(x=jx.with_values(n2), x_kv=jkv, is_causal=False, jagged=True,
                                     use_cache=use_cache, residual=h, kv_values=kv, proj_values=q2).values()
        n3, hr = hip_ops.rmsnorm_fork(h, norm.eps, norm.weight)
        fused = self._ff_residual(mlp, drop, n3, hr)
        if fused is not None:
            return jx.with_values(fused)
        y = mlp(n3)
        if drop.training and drop.p > 0 and hip_ops.dropout_fusable(hr) and hip_ops.dropout_fusable(y):
            return jx.with_values(hip_ops.dropout_add(hr, y, drop.p))
        return jx.with_values(hr + drop(y))

    def _pair_ok(self, n1, n2) -> bool:
        a, c = self.attention, self.cross_attention
        return (a.qkv.bias is None and c.q.bias is None and
                hip_ops.linear_pair_supported(n1, a.qkv.weight, n2, c.q.weight))

    def reset_kv_cache(self):
        raise NotImplementedError("KV Cache currently not supported")

    def apply_to_kv_cache(self, fn):
        raise NotImplementedError("KV Cache currently not supported")


class TransformerDecoder(nn.Module, KVCacheOpsMixin):
    def __init__(self, d_in: int, d_out: int, dropout: float, num_heads: int, n_layers: int,
                 do_cross_attn: bool = False, enable_kv_cache: bool = True) -> None:
        super().__init__()
        self.do_cross_attn = do_cross_attn
        self.layers = nn.ModuleList([
            TransformerBlock(d_in=d_in, d_out=d_out, dropout=dropout, num_heads=num_heads, qkv_bias=False,
                             do_cross_attn=do_cross_attn, enable_kv_cache=enable_kv_cache)
            for _ in range(n_layers)
        ])

    def forward(self, x: AttentionInput, padding_mask: Optional[Tensor] = None, is_causal: Optional[bool] = True,
                context: Optional[Tensor] = None, jagged: Optional[bool] = None) -> AttentionInput:
        if not jagged:
            raise Exception("Unjagged attention currently not supported.")
        h = as_jagged(x)
        ctx = as_jagged(context) if context is not None else None
        kvs = self._hoisted_kv(ctx)
        for i, layer in enumerate(self.layers):
            h = layer._forward_jagged(h, ctx, is_causal, kvs[i] if kvs is not None else None)
        return h if isinstance(x, Jagged) else _wrap_like(h.values(), x)

    def hoisted_kv_weights(self):
        """The cross-attention K/V weights _hoisted_kv concatenates (for the forward's weight split), or None."""
        if not (_HOIST_KV and self.do_cross_attn and len(self.layers) > 1):
            return None
        kvs = [layer.cross_attention.kv for layer in self.layers]
        return None if any(m.bias is not None for m in kvs) else [m.weight for m in kvs]

    def _hoisted_kv(self, ctx: Optional[Jagged]):
        """Every layer's cross-attention `kv(context)` as one GEMM over the concatenated K/V weights
        (they all project the same encoder output): hip_ops.hoisted_projection — one launch instead of
        one per layer forward, and in the backward one data-gradient GEMM (K = layers x 2 d_out) instead
        of per-layer GEMMs plus the adds of their context gradients. None when it does not apply."""
        if not (_HOIST_KV and self.do_cross_attn and ctx is not None and len(self.layers) > 1):
            return None
        kvs = [layer.cross_attention.kv for layer in self.layers]
        if any(m.bias is not None for m in kvs):
            return None
        return hip_ops.hoisted_projection(ctx.values(), [m.weight for m in kvs])


class TransformerEncoderDecoder(nn.Module, KVCacheOpsMixin):
    def __init__(self, d_in: int, d_out: int, dropout: float, num_heads: int, encoder_layers: int,
                 decoder_layers: int) -> None:
        super().__init__()
        self.encoder = TransformerDecoder(d_in=d_in, d_out=d_out, dropout=dropout, num_heads=num_heads,
                                          n_layers=encoder_layers, do_cross_attn=False, enable_kv_cache=False)
        self.decoder = TransformerDecoder(d_in=d_in, d_out=d_out, dropout=dropout, num_heads=num_heads,
                                          n_layers=decoder_layers, do_cross_attn=True, enable_kv_cache=False)
        self.layers = [self.encoder, self.decoder]
        self.cached_enc_output = None

    def forward(self, x: AttentionInput, padding_mask: Optional[Tensor] = None, context: Optional[Tensor] = None,
                jagged: Optional[bool] = None) -> AttentionInput:
        if self.cached_enc_output is None:
            context = self.encoder(context, padding_mask=padding_mask, is_causal=False, context=None, jagged=jagged)
            if not self.training:
                self.cached_enc_output = context
        else:
            context = self.cached_enc_output
        return self.decoder(x, padding_mask=None, is_causal=True, context=context, jagged=jagged)
