"""Weight-gradient GEMMs (dW += g^T x over many rows: the decoder's 11k-row context layers, C4's ~3k rows,
the RQ-VAE's 65,536 rows) under kernel policies, slab reduction included (accumulate, not deferred), each as a
hipGraph of 20 back-to-back calls. One JSON line per (shape, policy): the plan and the time per call.

  python tools/wgrad_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402


def main():
    from rqvae_hip import ops
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(0)
    shapes = [(1536, 512, 11332), (512, 512, 11332), (1024, 512, 11332), (512, 1024, 11332), (4096, 512, 11332),
              (1152, 384, 3200), (384, 1024, 3200), (1024, 384, 3200), (512, 768, 65536), (256, 512, 65536)]
    policies = [("default", 0), ("only64", ops.GEMM_ONLY_64), ("only128", ops.GEMM_ONLY_128),
                ("no_wide", ops.GEMM_NO_WIDE)]
    reps = 20
    for O, I, R in shapes:
        g = torch.randn(R, O, generator=gen, device=dev)
        x = torch.randn(R, I, generator=gen, device=dev)
        out = torch.zeros(O, I, device=dev)
        for pname, flags in policies:
            with ops.gemm_policy(flags):
                kern, S = ops.gemm_x3_choice(O, I, R, False, False, False, False)
                fn = lambda: ops.gemm_x3(g, False, x, False, O, I, R, out=out, accumulate=True)   # noqa: E731
                fn()
                torch.cuda.synchronize()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    for _ in range(reps):
                        fn()
            best = None
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                graph.replay()
                e1.record()
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) * 1000.0 / reps
                best = t if best is None else min(best, t)
            print(json.dumps({"O": O, "I": I, "rows": R, "policy": pname, "kernel": kern, "S": S,
                              "slab_MB": round(4 * O * I * S / 1e6, 1) if S > 1 else 0,
                              "us_per_call": round(best, 2)}), flush=True)
            del graph


if __name__ == "__main__":
    main()
