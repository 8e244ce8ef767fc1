#!/usr/bin/env python3
"""Short program for rocprofv3 --pmc passes: the fused quantize forward (rq_quantize_fwd) at the
bench workload (ML-32M: B=65,536, D=64, K=256, L=3, rotation trick), N launches, nothing else on
the GPU besides input setup. Run one counter group per process, e.g.

  rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rq_fwd -d out -o q -f csv -- python3 tools/pmc_quantize.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402

from rqvae_hip._lib import call, ptr, stream_handle  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    B, D, K, L = 65536, 64, 256, 3
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, D, generator=g, device=dev)
    x = x / x.norm(dim=1, keepdim=True)
    # codebooks = residual rows of other items (k-means-like)
    cbs = torch.randn(L, K, D, generator=g, device=dev)
    cbs = (cbs / cbs.norm(dim=2, keepdim=True)) * torch.tensor([1.0, 0.5, 0.25], device=dev).view(L, 1, 1)
    csq = (cbs * cbs).sum(-1).contiguous()
    ids = torch.empty(B, L, dtype=torch.int64, device=dev)
    emb, res = torch.empty(L, B, D, device=dev), torch.empty(L, B, D, device=dev)
    ql, es = torch.empty(B, device=dev), torch.empty(B, D, device=dev)
    for _ in range(n):
        call("rq_quantize_fwd", ptr(x), B, D, ptr(cbs), ptr(csq), K, L, 3, 0.25, ptr(ids), ptr(emb), ptr(res), ptr(ql),
             ptr(es), None, 0, stream_handle())
    torch.cuda.synchronize()
    print(f"pmc_quantize: {n} launches of rq_quantize_fwd at B={B} D={D} K={K} L={L}")


if __name__ == "__main__":
    main()
