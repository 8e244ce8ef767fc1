"""Split-bf16 GEMM launch time by operand form at the decoder's shapes (one process, HIP events, median of
interleaved rounds): does a pre-split operand (bf16 hi / lo planes produced upstream) beat an fp32 operand
split while staged, for the data- / weight-gradient pair and the forward projections? One JSON line per
(shape, form)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402

from rqvae_hip import ops  # noqa: E402


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


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    rows = 11264   # decoder Amazon context rows (bucketed)
    res = []
    # (name, O, I): qkv (A -> 3A), proj (A -> A), FF1 (A -> F), FF2 (F -> A), hoisted K/V (A -> 8 A)
    for name, O, I in (("qkv", 1536, 512), ("proj", 512, 512), ("ff1", 1024, 512), ("ff2", 512, 1024),
                       ("kv_hoist", 4096, 512)):
        x = torch.randn(rows, I, generator=g, device=dev)
        gy = torch.randn(rows, O, generator=g, device=dev)
        W = ops.split_bf16x3(torch.randn(O, I, generator=g, device=dev) * 0.05)
        xs, gs = ops.split_bf16x3(x), ops.split_bf16x3(gy)
        dw = torch.zeros(O, I, device=dev)
        for form, xa, ga in (("fp32", x, gy), ("split", xs, gs)):
            fwd = lambda: ops.gemm_x3(xa, True, W, True, rows, O, I)   # noqa: E731
            pair = lambda: ops.gemm_x3_pair(dict(a=ga, a_kcontig=True, b=W, b_kcontig=False, M=rows, N=I, K=O),  # noqa: E731
                                            dict(a=ga, a_kcontig=False, b=xa, b_kcontig=False, M=O, N=I, K=rows,
                                                 out=dw, accumulate=True))
            r = {"shape": name, "rows": rows, "O": O, "I": I, "form": form,
                 "fwd_us": round(timeit(fwd), 1), "fwd_kernel": ops.gemm_x3_choice(rows, O, I, form == "split", True,
                                                                                 True, True)[0],
                 "bwd_pair_us": round(timeit(pair), 1)}
            print(json.dumps(r), flush=True)
            res.append(r)
        split_cost = timeit(lambda: ops.split_bf16x3(gy))
        print(json.dumps({"shape": name, "split_gy_us": round(split_cost, 1),
                          "split_x_us": round(timeit(lambda: ops.split_bf16x3(x)), 1)}), flush=True)


if __name__ == "__main__":
    main()
