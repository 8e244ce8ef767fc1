"""Time single split-bf16 GEMM shapes (both operands pre-split, plain store) as a hipGraph of back-to-back
calls, under whichever library RQVAE_HIP_LIB names — for cross-process A/Bs of kernel builds (e.g. the wide
kernel's diagnostic builds). One JSON line per shape.

  RQVAE_HIP_LIB=build_ab/x.so python tools/gemm_shape_time.py [tag]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402

# (M, N, K, a_kcontig, b_kcontig): the RQ-VAE step's wide launches (forward / data grad / weight grad)
SHAPES = [(65536, 768, 512, True, True), (65536, 512, 768, True, True), (65536, 512, 512, True, False),
          (768, 512, 65536, False, False), (11332, 1024, 512, True, True)]
# the decoder's context-row launches on the 128-tile kernel: A fp32 (split while staged), B pre-split
DEC_SHAPES = [(11332, 1536, 512, True, True), (11332, 512, 1536, True, False), (11332, 1024, 512, True, True),
              (11332, 512, 1024, True, False)]


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    best = None
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1000.0 / reps
        best = t if best is None else min(best, t)
    return round(best, 2)


def main():
    from rqvae_hip import ops
    tag = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("RQVAE_HIP_LIB", "default")
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(0)
    for M, N, K, akc, bkc in SHAPES:
        a = ops.split_bf16x3(torch.randn((M, K) if akc else (K, M), generator=gen, device=dev))
        b = ops.split_bf16x3(torch.randn((N, K) if bkc else (K, N), generator=gen, device=dev) * 0.05)
        out = torch.zeros(M, N, device=dev)
        acc = M * N <= 1 << 20
        us = timed(lambda: ops.gemm_x3(a, akc, b, bkc, M, N, K, out=out if acc else None, accumulate=acc))
        kern, S = ops.gemm_x3_choice(M, N, K, True, True, akc, bkc, 0)
        print(json.dumps({"tag": tag, "M": M, "N": N, "K": K, "akc": akc, "bkc": bkc, "kernel": kern, "S": S,
                          "us": us, "tflops": round(2.0 * M * N * K / us / 1e6, 1)}), flush=True)
    for M, N, K, akc, bkc in DEC_SHAPES:
        a = torch.randn((M, K) if akc else (K, M), generator=gen, device=dev)
        b = ops.split_bf16x3(torch.randn((N, K) if bkc else (K, N), generator=gen, device=dev) * 0.05)
        us = timed(lambda: ops.gemm_x3(a, akc, b, bkc, M, N, K))
        kern, S = ops.gemm_x3_choice(M, N, K, False, True, akc, bkc, 0)
        print(json.dumps({"tag": tag, "M": M, "N": N, "K": K, "akc": akc, "bkc": bkc, "a": "fp32", "kernel": kern,
                          "S": S, "us": us, "tflops": round(2.0 * M * N * K / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
