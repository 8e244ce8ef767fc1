#!/usr/bin/env python3
"""Gumbel-softmax quantize (training, L2) fwd + bwd at the RQ-VAE ML-32M level shape (B=65,536, D=64, K=256):
HIP row kernels (rq_gumbel_softmax_fwd / _bwd + the codebook-gradient GEMMs) vs the torch composite of the
reference math, HIP events, same noise.   python tools/gumbel_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402


def main():
    import modules.quantize as mq
    from modules.quantize import Quantize, QuantizeForwardMode
    dev = torch.device("cuda", 0)
    B, D, K, T = 65536, 64, 256, 0.5
    torch.manual_seed(0)
    x = torch.randn(B, D, device=dev).requires_grad_(True)
    g = torch.randn(B, D, device=dev)
    for hip in (True, False, True, False):
        mq.GUMBEL_HIP = hip
        q = Quantize(D, K, do_kmeans_init=False, forward_mode=QuantizeForwardMode.GUMBEL_SOFTMAX).to(dev).train()

        def step():
            o = q(x, temperature=T)
            ((o.embeddings * g).sum() + o.loss.sum()).backward()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            step()
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"path": "hip" if hip else "composite", "B": B, "D": D, "K": K,
                          "ms_fwd_bwd": round(e0.elapsed_time(e1) / 10, 4)}), flush=True)


if __name__ == "__main__":
    main()
