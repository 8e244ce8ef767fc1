#!/usr/bin/env python3
"""Same-process A/B of the attention kernel families at the decoder's Amazon shapes, through the packed
autograd path the model uses (varlen_attention_packed: self-attention on a (T, 3A) qkv buffer, cross-
attention on q (Tq, A) + kv (Tk, 2A)); the LDS-DMA / few-query forms on and off alternately (rq_attn_dma_
enable), HIP events around `reps` forward and forward+backward passes, best of `rounds`.
   python3 tools/attn_ab2.py [reps] [rounds]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rq-vae-recommender_amd"))
from rqvae_hip import _lib, ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
g = np.random.Generator(np.random.PCG64(7))
B, H, hd, L1 = 256, 8, 64, 4
A = H * hd
lens = L1 * g.integers(2, 21, size=B) + 1
cu = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)])).to(dev)
T = int(lens.sum())
mx = int(lens.max())
qkv = torch.randn(T, 3 * A, device=dev, requires_grad=True)
nq = L1 + 1
cq = torch.arange(0, B + 1, device=dev, dtype=torch.int64) * nq
qc = torch.randn(B * nq, A, device=dev, requires_grad=True)
kv = torch.randn(T, 2 * A, device=dev, requires_grad=True)
qkv_f = torch.randn(B * nq, 3 * A, device=dev, requires_grad=True)
cases = {
    "enc_self": (lambda: ops.varlen_attention_packed(qkv, None, cu, cu, H, False, mx, mx), [qkv]),
    "cross": (lambda: ops.varlen_attention_packed(qc, kv, cq, cu, H, False, nq, mx), [qc, kv]),
    "dec_self": (lambda: ops.varlen_attention_packed(qkv_f, None, cq, cq, H, True, nq, nq), [qkv_f]),
}


def t(fn):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


lib = _lib.load()
res = {}
for r in range(rounds):
    for dma in (1, 0):
        lib.rq_attn_dma_enable(dma)
        for name, (fwd, ins) in cases.items():
            out = fwd()
            go = torch.randn_like(out)
            f_us = t(fwd)
            fb_us = t(lambda: torch.autograd.grad(fwd(), ins, go))
            key = (name, dma)
            best = res.get(key)
            if best is None or fb_us < best[1]:
                res[key] = (f_us, fb_us)
lib.rq_attn_dma_enable(1)
for (name, dma), (f_us, fb_us) in sorted(res.items()):
    print(json.dumps({"case": name, "dma": dma, "fwd_us": round(f_us, 1), "bwd_us": round(fb_us - f_us, 1),
                      "fwd_bwd_us": round(fb_us, 1)}), flush=True)
