#!/usr/bin/env python3
"""Ceiling probe for the decoder's context-row GEMMs: the split-bf16 product (hi.hi + hi.lo + lo.hi)
written as ONE bf16 GEMM over a tripled k axis (A' = [A_hi | A_hi | A_lo], B' = [B_hi | B_lo | B_hi])
on the library (torch.matmul -> hipBLASLt, fp32 accumulate), next to rq_gemm_bf16x3 at the same
shape (fp32 A / split B, and both split). Prints one JSON line per shape: device us per launch
(HIP events over `reps` launches) and fp32-matmul TFLOP/s (2 M N K / t).

  python tools/lib_bf16_probe.py [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402

from rqvae_hip import ops  # noqa: E402

# (M, N, K, a_kc, b_kc): decoder Amazon context rows (11,264 = 44 x 256), forward / dgrad / wgrad forms
SHAPES = [
    (11264, 1536, 512, 1, 1),    # qkv forward
    (11264, 512, 1536, 1, 0),    # qkv dgrad
    (11264, 1024, 512, 1, 1),    # fc1 forward
    (11264, 512, 1024, 1, 0),    # fc1 dgrad / fc2 forward
    (11264, 512, 512, 1, 1),     # proj forward
    (11264, 4096, 512, 1, 1),    # hoisted cross K/V forward
    (11264, 512, 4096, 1, 0),    # hoisted cross K/V dgrad
    (1536, 512, 11264, 0, 0),    # qkv wgrad
    (65536, 768, 512, 1, 1),     # RQ-VAE decoder last layer forward (reference point)
]


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for M, N, K, akc, bkc in SHAPES:
        a = torch.randn((M, K) if akc else (K, M), generator=g, device=dev)
        b = torch.randn((N, K) if bkc else (K, N), generator=g, device=dev)
        am = a if akc else a.t()   # (M, K) logical
        bm = b if bkc else b.t()   # (N, K) logical
        ah = am.to(torch.bfloat16)
        al = (am - ah.float()).to(torch.bfloat16)
        bh = bm.to(torch.bfloat16)
        bl = (bm - bh.float()).to(torch.bfloat16)
        A3 = torch.cat([ah, ah, al], dim=1).contiguous()          # (M, 3K)
        B3 = torch.cat([bh, bl, bh], dim=1).contiguous()          # (N, 3K)
        out = torch.empty(M, N, device=dev, dtype=torch.float32)
        flops = 2.0 * M * N * K
        r = {"shape": [M, N, K, akc, bkc]}
        # library bf16 GEMM over 3K, bf16 output (fp32 accumulate inside) and fp32-out variant
        t = timed(lambda: torch.matmul(A3, B3.t()), reps)
        r["lib_bf16_3k_us"] = round(t, 1)
        r["lib_bf16_3k_tflops"] = round(flops / (t * 1e-6) / 1e12, 1)
        t = timed(lambda: torch.mm(am, bm.t(), out=out), reps)
        r["lib_fp32_us"] = round(t, 1)
        # this build's split-bf16 kernel: fp32 A, split B; and both split
        bs = ops.split_bf16x3(b)
        t = timed(lambda: ops.gemm_x3(a, bool(akc), bs, bool(bkc), M, N, K), reps)
        r["x3_fp32A_splitB_us"] = round(t, 1)
        r["x3_fp32A_splitB_tflops"] = round(flops / (t * 1e-6) / 1e12, 1)
        asp = ops.split_bf16x3(a)
        t = timed(lambda: ops.gemm_x3(asp, bool(akc), bs, bool(bkc), M, N, K), reps)
        r["x3_split_us"] = round(t, 1)
        r["x3_split_tflops"] = round(flops / (t * 1e-6) / 1e12, 1)
        r["plan_split"] = ops.gemm_x3_choice(M, N, K, True, True, bool(akc), bool(bkc), 0)
        print(json.dumps(r), flush=True)
        del a, b, A3, B3, out, bs, asp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
