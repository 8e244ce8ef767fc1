#!/usr/bin/env python3
"""Would one launch holding a data-gradient GEMM and its weight-gradient GEMM beat two launches? Times the
decoder's (dgrad, wgrad) pairs back to back on one stream and concurrently on two streams (HIP events,
`reps` repetitions each, plain eager launches): the concurrent time bounds what a paired launch could gain
from filling the chip with both problems and sharing one launch.

  python tools/pair_probe.py [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402

from rqvae_hip import ops  # noqa: E402

# (rows, in, out): the decoder's future-token rows (Amazon 1,280 / ML-32M B=8: 40) and context rows
PAIRS = [(1280, 512, 512), (1280, 512, 1536), (1280, 1024, 512), (40, 384, 384), (40, 384, 1152),
         (11264, 512, 1536), (11264, 512, 512), (11264, 1024, 512)]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for rows, I, O in PAIRS:
        gr = torch.randn(rows, O, generator=g, device=dev)          # output gradient (fp32)
        x = torch.randn(rows, I, generator=g, device=dev)            # layer input (fp32)
        W = ops.split_bf16x3(torch.randn(O, I, generator=g, device=dev))
        dW = torch.zeros(O, I, device=dev)

        def dgrad():
            return ops.gemm_x3(gr, True, W, False, rows, I, O)

        def wgrad():
            return ops.gemm_x3(gr, False, x, False, O, I, rows, out=dW, accumulate=True)

        def seq():
            dgrad()
            wgrad()

        def conc():
            cur = torch.cuda.current_stream()
            s1.wait_stream(cur)
            s2.wait_stream(cur)
            with torch.cuda.stream(s1):
                dgrad()
            with torch.cuda.stream(s2):
                wgrad()
            cur.wait_stream(s1)
            cur.wait_stream(s2)

        res = {"rows": rows, "in": I, "out": O}
        for name, fn in (("dgrad", dgrad), ("wgrad", wgrad), ("sequential", seq), ("concurrent", conc)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                fn()
            b.record()
            torch.cuda.synchronize()
            res[name + "_us"] = round(a.elapsed_time(b) / reps * 1e3, 1)
        res["dgrad_plan"] = ops.gemm_x3_choice(rows, I, O, False, True, True, False)
        res["wgrad_plan"] = ops.gemm_x3_choice(O, I, rows, False, False, False, False)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
