"""Paired data + weight gradient launches (rq_gemm_bf16x3_pair) of the decoder's context-row Linears with the
weight gradient's split-K count forced (RQ_GEMM_SPLIT per descriptor), its deferred slab reduction flushed
inside the timed graph: does a pair want fewer weight-gradient slabs than the call planned alone? One JSON
line per (shape, S).

  python tools/pair_split_probe.py [future | hoisted]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402


def timed(fn, reps=10):
    from rqvae_hip import ops
    fn()
    ops.flush_reductions()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
        ops.flush_reductions()
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
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(0)
    # (rows, O, I, data-grad A split?): Amazon qkv / MLP up / MLP down / proj; C4 context qkv / up
    shapes = [(11332, 1536, 512, False), (11332, 1024, 512, True), (11332, 512, 1024, False), (11332, 512, 512, False),
              (3200, 1152, 384, False), (3200, 1024, 384, True)]
    if len(sys.argv) > 1 and sys.argv[1] == "hoisted":   # the decoder's hoisted cross-attention K/V backward
        shapes = [(11332, 4096, 512, False), (3200, 3072, 384, False)]
    if len(sys.argv) > 1 and sys.argv[1] == "future":   # the future-token rows: Amazon 1,280, C4 40
        shapes = [(1280, 1536, 512, False), (1280, 512, 512, False), (1280, 1024, 512, True), (1280, 512, 1024, False),
                  (40, 1152, 384, False), (40, 384, 384, False), (40, 1024, 384, True), (40, 384, 1024, False)]
    for R, O, I, gsplit in shapes:
        g = torch.randn(R, O, generator=gen, device=dev)
        ga = ops.split_bf16x3(g) if gsplit else g
        x = torch.randn(R, I, generator=gen, device=dev)
        W = ops.split_bf16x3(torch.randn(O, I, generator=gen, device=dev) * 0.05)
        dW = torch.zeros(O, I, device=dev)
        _, s_auto = ops.gemm_x3_choice(O, I, R, gsplit, False, False, False)
        for S in ([0, 1, 2, 3, 4, 5, 6, 8] if len(sys.argv) > 1 and sys.argv[1] == "hoisted" else
                  [0, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32]):
            f = ops.gemm_split(S) if S else None

            def fn():
                ops.gemm_x3_pair(dict(a=ga, a_kcontig=True, b=W, b_kcontig=False, M=R, N=I, K=O),
                                 dict(a=ga, a_kcontig=False, b=x, b_kcontig=False, M=O, N=I, K=R, out=dW,
                                      accumulate=True, defer=True, flags=f))
            print(json.dumps({"rows": R, "O": O, "I": I, "S": S or s_auto, "planned": S == 0, "us": timed(fn)}),
                  flush=True)


if __name__ == "__main__":
    main()
