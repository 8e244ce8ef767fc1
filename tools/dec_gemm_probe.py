#!/usr/bin/env python3
"""Decoder context-row GEMM shapes (Amazon: ~11,332 rows): device time of the production operand form
(fp32 activation x split weight, 128-tile kernel with on-the-fly conversion) against split activations on
the 128-tile kernel, the wide kernel, and a 'wide + tail' composition (the wide kernel over the largest
row block that fills at most one round of 256 wide tiles, the 128-tile kernel over the remaining rows).
   python3 tools/dec_gemm_probe.py [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rq-vae-recommender_amd"))
import torch  # noqa: E402

from rqvae_hip import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
CASES = [(11332, 1536, 512, True, True, "qkv fwd"), (11332, 1024, 512, True, True, "ff1/kv fwd"),
         (11332, 512, 1024, True, True, "ff2 fwd"), (11332, 512, 512, True, True, "proj fwd"),
         (11332, 512, 1536, True, False, "qkv dgrad"), (11332, 512, 1024, True, False, "kv/ff1 dgrad"),
         (11332, 512, 512, True, False, "proj dgrad"), (11332, 1024, 512, True, False, "ff2 dgrad"),
         (1536, 512, 11332, False, False, "qkv wgrad"), (1024, 512, 11332, False, False, "ff1/kv wgrad"),
         (512, 512, 11332, False, False, "proj wgrad"), (512, 1024, 11332, False, False, "ff2 wgrad")]


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
for M, N, K, akc, bkc, tag in CASES:
    a = torch.randn((M, K) if akc else (K, M), device=dev)
    b = torch.randn((N, K) if bkc else (K, N), device=dev)
    sa, sb = ops.split_bf16x3(a), ops.split_bf16x3(b)
    res = {}
    ops.gemm_x3w_enable(True)
    res["prod_fp32A"] = timed(lambda: ops.gemm_x3(a, akc, sb, bkc, M, N, K))
    if not akc:   # weight grads: both operands fp32 in production
        res["prod_fp32AB"] = timed(lambda: ops.gemm_x3(a, akc, b, bkc, M, N, K))
    ops.gemm_x3w_enable(False)
    res["x3_split"] = timed(lambda: ops.gemm_x3(sa, akc, sb, bkc, M, N, K))
    ops.gemm_x3w_enable(2)
    res["wide_split"] = timed(lambda: ops.gemm_x3(sa, akc, sb, bkc, M, N, K))
    if akc:
        tiles_n = (N + 255) // 256
        m1 = min(M // 256, 256 // tiles_n) * 256
        if 0 < m1 < M:
            C = torch.empty((M, N), device=dev)
            sa1 = ops.Split(sa.hi[:m1], sa.lo[:m1])
            sa2 = ops.Split(sa.hi[m1:], sa.lo[m1:])

            def hybrid():
                ops.gemm_x3w_enable(2)
                ops.gemm_x3(sa1, True, sb, bkc, m1, N, K, out=C[:m1])
                ops.gemm_x3w_enable(False)
                ops.gemm_x3(sa2, True, sb, bkc, M - m1, N, K, out=C[m1:])
            res[f"wide{m1}+tail"] = timed(hybrid)
    ops.gemm_x3w_enable(True)
    print(json.dumps({"case": tag, "M": M, "N": N, "K": K, **{k: round(v, 2) for k, v in res.items()},
                      "tflops_best": round(2.0 * M * N * K / min(res.values()) / 1e6, 1)}), flush=True)
    del a, b, sa, sb
