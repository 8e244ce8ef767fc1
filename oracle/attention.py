"""Varlen (jagged) scaled-dot-product attention, forward and backward — numpy float64.

Reference: modules/transformer/attention.py:113-124 (Attend.jagged_forward ->
F.scaled_dot_product_attention on NJT q/k/v (B, H, j, hd), dropout 0, scale 1/sqrt(hd),
is_causal top-left aligned). Computed in float64 as the checker for float32 kernels.
Test infrastructure only.
"""
import numpy as np


def _seg(cu, b):
    return int(cu[b]), int(cu[b + 1])


def attn_fwd(q, k, v, cu_q, cu_k, causal, scale=None):
    """q: (Tq, H, hd), k/v: (Tk, H, hd) packed; cu_*: (B+1,) offsets. Returns out (Tq,H,hd), lse (H,Tq)."""
    q64, k64, v64 = (a.astype(np.float64) for a in (q, k, v))
    Tq, H, hd = q.shape
    scale = 1.0 / np.sqrt(hd) if scale is None else scale
    out = np.zeros((Tq, H, hd))
    lse = np.zeros((H, Tq))
    for b in range(len(cu_q) - 1):
        q0, q1 = _seg(cu_q, b)
        k0, k1 = _seg(cu_k, b)
        if q1 == q0:
            continue
        for h in range(H):
            s = q64[q0:q1, h] @ k64[k0:k1, h].T * scale
            if causal:
                s = np.where(np.tril(np.ones_like(s, dtype=bool)), s, -np.inf)
            m = s.max(1, keepdims=True)
            m = np.where(np.isfinite(m), m, 0.0)
            p = np.exp(s - m)
            l = p.sum(1, keepdims=True)
            out[q0:q1, h] = (p / np.where(l > 0, l, 1.0)) @ v64[k0:k1, h]
            lse[h, q0:q1] = (m + np.log(np.where(l > 0, l, 1.0)))[:, 0]
    return out, lse


def attn_bwd(q, k, v, dout, cu_q, cu_k, causal, scale=None):
    """Returns dq, dk, dv (same packed layouts) for attn_fwd."""
    q64, k64, v64, do64 = (a.astype(np.float64) for a in (q, k, v, dout))
    Tq, H, hd = q.shape
    scale = 1.0 / np.sqrt(hd) if scale is None else scale
    dq, dk, dv = np.zeros_like(q64), np.zeros_like(k64), np.zeros_like(v64)
    for b in range(len(cu_q) - 1):
        q0, q1 = _seg(cu_q, b)
        k0, k1 = _seg(cu_k, b)
        if q1 == q0:
            continue
        for h in range(H):
            s = q64[q0:q1, h] @ k64[k0:k1, h].T * scale
            if causal:
                s = np.where(np.tril(np.ones_like(s, dtype=bool)), s, -np.inf)
            s = s - s.max(1, keepdims=True)
            p = np.exp(s)
            p /= p.sum(1, keepdims=True)
            do = do64[q0:q1, h]
            dv[k0:k1, h] += p.T @ do
            dp = do @ v64[k0:k1, h].T
            ds = p * (dp - (dp * p).sum(1, keepdims=True))
            dq[q0:q1, h] += ds @ k64[k0:k1, h] * scale
            dk[k0:k1, h] += ds.T @ q64[q0:q1, h] * scale
    return dq, dk, dv
