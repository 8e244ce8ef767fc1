#!/usr/bin/env python3
"""A/B of the split-bf16 GEMM kernels on the RQ-VAE (and decoder) shapes: the wide 256-tile kernel
vs the 128-tile kernel, both operands pre-split, HIP events around `reps` back-to-back launches.
Prints one JSON line per (shape, layout, kernel): us per launch and fp32-equivalent TFLOP/s.
   python3 tools/gemm_ab.py [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rq-vae-recommender_amd"))
import torch  # noqa: E402

from rqvae_hip import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
# (M, N, K, a_kc, b_kc, tag): the RQ-VAE MLP chain at B = 65536 (fwd / dgrad / wgrad) + decoder rows
CASES = [
    (65536, 512, 768, True, True, "enc0 fwd"), (65536, 768, 512, True, False, "enc0 dgrad"),
    (512, 768, 65536, False, False, "enc0 wgrad"),
    (65536, 256, 512, True, True, "enc1 fwd"), (65536, 512, 256, True, False, "enc1 dgrad"),
    (256, 512, 65536, False, False, "enc1 wgrad"),
    (65536, 768, 512, True, True, "dec3 fwd"), (65536, 512, 768, True, False, "dec3 dgrad"),
    (768, 512, 65536, False, False, "dec3 wgrad"),
    (65536, 512, 256, True, True, "dec2 fwd"), (65536, 256, 512, True, False, "dec2 dgrad"),
    (512, 256, 65536, False, False, "dec2 wgrad"),
    (20480, 1536, 512, True, True, "decoder qkv fwd"), (20480, 1024, 512, True, True, "decoder ff fwd"),
    (1536, 512, 20480, False, False, "decoder qkv wgrad"),
    (11332, 1536, 512, True, True, "dec-ctx qkv fwd"), (11332, 1024, 512, True, True, "dec-ctx ff1 fwd"),
    (11332, 512, 1024, True, True, "dec-ctx ff2 fwd"), (11332, 512, 1536, True, False, "dec-ctx qkv dgrad"),
    (11332, 512, 512, True, True, "dec-ctx out fwd"), (1536, 512, 11332, False, False, "dec-ctx qkv wgrad"),
    (1024, 512, 11332, False, False, "dec-ctx ff1 wgrad"), (512, 512, 11332, False, False, "dec-ctx out wgrad"),
]


def timed(fn):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


extra = os.environ.get("GEMM_AB_EXTRA")        # "M,N,K,akc,bkc;..." appended as 'extra' cases
if extra:
    for e in extra.split(";"):
        M_, N_, K_, a_, b_ = (int(v) for v in e.split(","))
        CASES.append((M_, N_, K_, bool(a_), bool(b_), f"extra {M_}x{N_}x{K_}:{a_}{b_}"))
torch.manual_seed(0)
only = os.environ.get("GEMM_AB_CASES")          # comma-separated substrings of the case tags
kernels = os.environ.get("GEMM_AB_KERNELS", "wide,x3").split(",")
for M, N, K, akc, bkc, tag in CASES:
    if only and not any(o in tag for o in only.split(",")):
        continue
    a = torch.randn((M, K) if akc else (K, M), device=dev)
    b = torch.randn((N, K) if bkc else (K, N), device=dev)
    sa, sb = ops.split_bf16x3(a), ops.split_bf16x3(b)
    out = {}
    for wide in [k == "wide" for k in kernels]:
        ops.gemm_x3w_enable(2 if wide else False)   # forced either way
        kern, S = ops.gemm_x3_choice(M, N, K, True, True, akc, bkc)
        us = timed(lambda: ops.gemm_x3(sa, akc, sb, bkc, M, N, K))
        out[kern] = us
        print(json.dumps({"case": tag, "M": M, "N": N, "K": K, "kernel": kern, "splits": S, "us": round(us, 2),
                          "tflops": round(2.0 * M * N * K / us / 1e6, 1)}), flush=True)
    ops.gemm_x3w_enable(True)
    print(json.dumps({"case": tag, "model_picks": ops.gemm_x3_choice(M, N, K, True, True, akc, bkc)[0],
                      "measured_best": min(out, key=out.get)}), flush=True)
    del a, b, sa, sb
