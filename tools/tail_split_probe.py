#!/usr/bin/env python3
"""Tile-quantisation probe for the 128-tile split-bf16 GEMM at the decoder's context-row shapes: one call
(rq_gemm_bf16x3_run over all M rows) against a paired launch of the rows that fill whole rounds of
resident workgroups (unsplit) and the remaining tail rows split-K S ways (rq_gemm_bf16x3_pair; the tail's
slab reduction follows in the same call). Each variant timed as a hipGraph of 20 calls; results compared
(the unsplit rows bitwise, the tail within split-K rounding). One JSON line per (shape, variant).
    python3 tools/tail_split_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402

from rqvae_hip import ops  # noqa: E402


def graph_ms(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / reps)
    return best * 1e3


def main():
    dev = torch.device("cuda", 0)
    slots = 2 * torch.cuda.get_device_properties(dev).multi_processor_count
    # (M, N, K, a fp32 k-contig?) — Amazon context rows (11,332 valid, bucketed rows vary)
    shapes = [(11332, 1536, 512), (11332, 1024, 512), (11332, 512, 1024), (11332, 512, 512), (11520, 1536, 512)]
    g = torch.Generator(device=dev).manual_seed(0)
    for M, N, K in shapes:
        a = torch.randn(M, K, device=dev, generator=g)
        w = ops.split_bf16x3(torch.randn(N, K, device=dev, generator=g) * 0.05)
        tiles_n = -(-N // 128)
        out = {}

        def full():
            out["full"] = ops.gemm_x3(a, True, w, True, M, N, K)
        res = {"M": M, "N": N, "K": K, "tiles": -(-M // 128) * tiles_n, "slots": slots}
        res["full_us"] = round(graph_ms(full), 2)
        ref = out["full"].clone()
        rounds = (-(-M // 128) * tiles_n) // slots
        m1 = (rounds * slots // tiles_n) * 128
        if 0 < m1 < M:
            for S in (2, 4, 8):
                C = torch.empty(M, N, device=dev)

                def pair():
                    s1 = dict(a=a[:m1], a_kcontig=True, b=w, b_kcontig=True, M=m1, N=N, K=K, out=C[:m1])
                    s2 = dict(a=a[m1:], a_kcontig=True, b=w, b_kcontig=True, M=M - m1, N=N, K=K, out=C[m1:],
                              flags=ops.gemm_split(S))
                    ops.gemm_x3_pair(s1, s2)
                t = graph_ms(pair)
                res[f"pair_S{S}_us"] = round(t, 2)
                res["m1"] = m1
                res[f"pair_S{S}_head_bitwise"] = bool(torch.equal(C[:m1], ref[:m1]))
                res[f"pair_S{S}_tail_maxrel"] = float(((C[m1:] - ref[m1:]).abs().max() / ref.abs().max()).item())
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
