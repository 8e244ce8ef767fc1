"""Where does the wide split-bf16 GEMM (gemm_x3w_kernel, 256 x 256 tiles) lose its time? Launch time of the
plain-epilogue forward form (pre-split A and W, RQ_GEMM_FORCE_WIDE) over a sweep of K at the RQ-VAE's
65,536 rows (slope = k-loop rate, intercept = per-tile prologue + epilogue) and over M at K = 512 (rounds
of 256 workgroups). One JSON line per point: us, TFLOP/s, fraction of the 833 TF split ceiling."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402

from rqvae_hip import ops  # noqa: E402

PEAK = 2500.0 / 3


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def point(M, N, K, g, dev, tag):
    x = ops.split_bf16x3(torch.randn(M, K, generator=g, device=dev))
    w = ops.split_bf16x3(torch.randn(N, K, generator=g, device=dev) * 0.05)
    with ops.gemm_policy(ops.GEMM_FORCE_WIDE):
        kern = ops.gemm_x3_choice(M, N, K, True, True, True, True)[0]
        us = timeit(lambda: ops.gemm_x3(x, True, w, True, M, N, K))
    tf = 2.0 * M * N * K / us / 1e6
    r = {"sweep": tag, "M": M, "N": N, "K": K, "kernel": kern, "us": round(us, 2), "tflops": round(tf, 1),
         "frac": round(tf / PEAK, 3), "tiles": (M // 256) * (N // 256)}
    print(json.dumps(r), flush=True)
    del x, w


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for N in (768, 512):
        for K in (256, 512, 1024, 2048, 4096):
            point(65536, N, K, g, dev, "K")
    for M in (16384, 32768, 65536, 131072, 262144):
        point(M, 768, 512, g, dev, "M")


if __name__ == "__main__":
    main()
