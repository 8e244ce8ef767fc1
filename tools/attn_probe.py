#!/usr/bin/env python3
"""Varlen attention fwd / bwd timing at the decoder configs' shapes (HIP events, one process).

  Amazon:  B=256 sequences, ctx len 4*U{2..20}+1 (<= 81), H=8, hd=64 (attn_dim 512)
  ML-32M:  B=64 sequences,  ctx len 4*U{2..200}+1 (<= 801), H=6, hd=64 (attn_dim 384)
  C5:      B=64 sequences,  ctx len 5*U{2..256}+1 (<= 1281), H=8, hd=64 (DA dims, L=4)
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rq-vae-recommender_amd"))
from rqvae_hip import ops  # noqa: E402


def t(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def case(name, B, H, hd, max_items, dev, L1=4, cross=False):
    g = np.random.Generator(np.random.PCG64(7))
    lens = L1 * g.integers(2, max_items + 1, size=B) + 1
    cu = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)])).to(dev)
    T = int(lens.sum())
    A = H * hd
    qkv = torch.randn(T, 3 * A, device=dev, requires_grad=True)
    q, k, v = qkv[:, :A], qkv[:, A:2 * A], qkv[:, 2 * A:]
    mx = int(lens.max())
    fwd = lambda: ops.varlen_attention(q, k, v, cu, cu, H, False, mx, mx)  # noqa: E731
    if cross:   # decoder cross-attention: L+2 future queries per sequence x its context keys
        nq = L1 + 1
        cq = torch.arange(0, B + 1, device=dev, dtype=torch.int64) * nq
        qc = torch.randn(B * nq, A, device=dev, requires_grad=True)
        fwd = lambda: ops.varlen_attention(qc, k, v, cq, cu, H, False, nq, mx)  # noqa: E731
        lens = np.sqrt(nq * lens.astype(np.float64))   # FLOPs ~ nq * n
    out = fwd()
    go = torch.randn_like(out)
    fb = lambda: torch.autograd.grad(fwd(), qkv, go)  # noqa: E731
    if cross:
        fb = lambda: torch.autograd.grad(fwd(), (qc, qkv), go)  # noqa: E731
    fl = 4.0 * hd * H * float((lens.astype(np.float64) ** 2).sum())
    for fused in (True, False):
        ops.ATTN_FUSED_BWD = fused
        ms_f, ms_fb = t(fwd), t(fb)
        print(json.dumps(dict(case=name, fused_bwd=fused, tokens=T, max_len=mx, fwd_ms=round(ms_f, 4),
                              fwd_bwd_ms=round(ms_fb, 4), bwd_ms=round(ms_fb - ms_f, 4),
                              fwd_tflops=round(fl / ms_f / 1e9, 1), bwd_tflops=round(2 * fl / (ms_fb - ms_f) / 1e9, 1))),
              flush=True)
    ops.ATTN_FUSED_BWD = True


def main():
    dev = torch.device("cuda", 0)
    if len(sys.argv) > 1:   # A/B: time an alternative build of the library
        from rqvae_hip import _lib
        _lib._lib = _lib.load(sys.argv[1])
        print(json.dumps(dict(lib=sys.argv[1])))
    case("amazon", 256, 8, 64, 20, dev)
    case("ml32m", 64, 6, 64, 200, dev)
    case("c5", 64, 8, 64, 256, dev, L1=5)
    case("amazon_cross", 256, 8, 64, 20, dev, cross=True)
    case("ml32m_cross", 64, 6, 64, 200, dev, cross=True)
    case("c5_cross", 64, 8, 64, 256, dev, L1=5, cross=True)


if __name__ == "__main__":
    main()
