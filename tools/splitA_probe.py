"""Forward split-bf16 GEMMs of the decoder's RMSNorm-fed projections with the activation operand fp32 (split
while staged, the current form) vs already split into bf16 planes (what a norm kernel could emit at the same
bytes), plus the paired backward (data + weight gradient) that reads the activation as its B operand. Each as
a hipGraph of 20 back-to-back calls. One JSON line per (shape, form).

  python tools/splitA_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    best = None
    for _ in range(3):
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
    # (rows, out, in, epilogue): Amazon context qkv / MLP up, future qkv / q / up; C4 context qkv / up
    shapes = [(11520, 1536, 512, ops.EPI_STORE), (11520, 1024, 512, ops.EPI_SILU_FWD), (1280, 1536, 512, ops.EPI_STORE),
              (1280, 512, 512, ops.EPI_STORE), (1280, 1024, 512, ops.EPI_SILU_FWD), (4608, 1152, 384, ops.EPI_STORE),
              (4608, 1024, 384, ops.EPI_SILU_FWD)]
    for M, O, I, epi in shapes:
        x = torch.randn(M, I, generator=gen, device=dev)
        xs = ops.split_bf16x3(x)
        W = ops.split_bf16x3(torch.randn(O, I, generator=gen, device=dev) * 0.05)
        g = torch.randn(M, O, generator=gen, device=dev)
        dW = torch.zeros(O, I, device=dev)
        row = {"M": M, "O": O, "I": I, "epi": epi}
        for name, a, sp in (("fp32", x, False), ("split", xs, True)):
            row["fwd_" + name] = timed(lambda: ops.gemm_x3(a, True, W, True, M, O, I, epi, p=0.1, seed=1))
            row["fwd_kernel_" + name] = ops.gemm_x3_choice(M, O, I, sp, True, True, True, epi)
            row["bwd_" + name] = timed(lambda: ops.gemm_x3_pair(
                dict(a=g, a_kcontig=True, b=W, b_kcontig=False, M=M, N=I, K=O),
                dict(a=g, a_kcontig=False, b=a, b_kcontig=False, M=O, N=I, K=M, out=dW, accumulate=True)))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
