#!/usr/bin/env python3
"""fp32 GEMM shapes of the RQ-VAE ML-32M train step (B=65536, 768->[512,256,128]->64 and the
mirror decoder): forward (x @ W^T), data grad (g @ W) and weight grad (g^T @ x), timed under
hipBLASLt and rocBLAS. Prints one JSON line per (shape, op, backend)."""
import json
import os
import sys

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


def main():
    dev = torch.device("cuda", 0)
    B = 65536
    dims = [(768, 512), (512, 256), (256, 128), (128, 64), (64, 128), (128, 256), (256, 512), (512, 768)]
    tot = {}
    for lib in ("cublaslt", "cublas"):
        torch.backends.cuda.preferred_blas_library(lib)
        tot[lib] = 0.0
        for (i, o) in dims:
            x = torch.randn(B, i, device=dev)
            w = torch.randn(o, i, device=dev)
            bias = torch.randn(o, device=dev)
            g = torch.randn(B, o, device=dev)
            fl = 2.0 * B * i * o
            for name, fn in (("fwd", lambda: torch.addmm(bias, x, w.t())), ("dgrad", lambda: g @ w),
                             ("wgrad", lambda: g.t() @ x)):
                ms = t(fn)
                tot[lib] += ms
                print(json.dumps(dict(lib=lib, shape=[B, i, o], op=name, ms=round(ms, 4),
                                      tflops=round(fl / ms / 1e9, 1))), flush=True)
    tot["rq_wgrad"] = 0.0
    for (i, o) in dims:
        x = torch.randn(B, i, device=dev)
        g = torch.randn(B, o, device=dev)
        ms = t(lambda: ops.linear_wgrad(g, x, False))
        tot["rq_wgrad"] += ms
        print(json.dumps(dict(lib="rq_linear_wgrad", shape=[B, i, o], op="wgrad", ms=round(ms, 4),
                              tflops=round(2.0 * B * i * o / ms / 1e9, 1))), flush=True)
    print(json.dumps(dict(total_ms=tot)))


if __name__ == "__main__":
    main()
