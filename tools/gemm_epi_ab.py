#!/usr/bin/env python3
"""Wide (256-tile) vs 128-tile split-bf16 GEMM on the RQ-VAE step's fused-epilogue launches (SiLU fwd
with dropout off / SiLU' bwd reading Z and emitting split planes), both operands pre-split, forced either
way; HIP events around `reps` back-to-back launches.   python3 tools/gemm_epi_ab.py [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rq-vae-recommender_amd"))
import torch  # noqa: E402

from rqvae_hip import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
B = 65536
CASES = [   # (M, N, K, a_kc, b_kc, epilogue, tag)
    (B, 512, 768, True, True, ops.EPI_SILU_FWD, "enc0 fwd silu"), (B, 256, 512, True, True, ops.EPI_SILU_FWD, "enc1 fwd silu"),
    (B, 256, 128, True, True, ops.EPI_SILU_FWD, "dec1 fwd silu"), (B, 512, 256, True, True, ops.EPI_SILU_FWD, "dec2 fwd silu"),
    (B, 768, 512, True, True, ops.EPI_STORE, "dec3 fwd"),
    (B, 512, 768, True, False, ops.EPI_SILU_BWD, "dec3 dgrad silu'"), (B, 256, 512, True, False, ops.EPI_SILU_BWD, "dec2 dgrad silu'"),
    (B, 256, 128, True, False, ops.EPI_SILU_BWD, "enc2 dgrad silu'"), (B, 512, 256, True, False, ops.EPI_SILU_BWD, "enc1 dgrad silu'"),
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


torch.manual_seed(0)
for M, N, K, akc, bkc, epi, tag in CASES:
    a = torch.randn((M, K) if akc else (K, M), device=dev)
    b = torch.randn((N, K) if bkc else (K, N), device=dev)
    z = torch.randn((M, N), device=dev) if epi == ops.EPI_SILU_BWD else None
    sa, sb = ops.split_bf16x3(a), ops.split_bf16x3(b)
    out = {}
    for mode in ("model", "wide", "x3"):
        ops.gemm_x3w_enable({"model": True, "wide": 2, "x3": False}[mode])
        kern, S = ops.gemm_x3_choice(M, N, K, True, True, akc, bkc, epi)
        us = timed(lambda: ops.gemm_x3(sa, akc, sb, bkc, M, N, K, epilogue=epi, Z=z))
        out[mode] = (kern, S, round(us, 2))
    ops.gemm_x3w_enable(True)
    print(json.dumps({"case": tag, "M": M, "N": N, "K": K, "epi": epi, **{k: v for k, v in out.items()},
                      "tflops_model": round(2.0 * M * N * K / out["model"][2] / 1e6, 1)}), flush=True)
    del a, b, sa, sb, z
