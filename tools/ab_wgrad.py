#!/usr/bin/env python3
"""In-process A/B of rq_linear_wgrad between the current library and an older build of the same
entry point (a standalone .so of a previous linear.hip), interleaved rounds, HIP events.

  python tools/ab_wgrad.py tools/_ab_wgrad_old.so
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402

from rqvae_hip import _lib  # noqa: E402
from rqvae_hip._lib import stream_handle  # noqa: E402

SIG = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
       ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]


def bind(lib):
    f = lib.rq_linear_wgrad
    f.argtypes, f.restype = SIG, ctypes.c_int
    w = lib.rq_linear_wgrad_workspace
    w.argtypes, w.restype = [ctypes.c_int64] * 3, ctypes.c_size_t
    return f, w


def main():
    dev = torch.device("cuda", 0)
    arms = {"new": bind(_lib.load()), "old": bind(ctypes.CDLL(os.path.abspath(sys.argv[1])))}
    dims = [768, 512, 256, 128, 64]
    cases = [(65536, o, i) for i, o in zip(dims[:-1], dims[1:])] + [(65536, i, o) for i, o in zip(dims[:-1], dims[1:])]
    tot = {a: 0.0 for a in arms}
    for (N, O, I) in cases:
        g = torch.Generator(device=dev).manual_seed(N + O + I)
        gy = torch.randn(N, O, generator=g, device=dev)
        x = torch.randn(N, I, generator=g, device=dev)
        outs, t = {}, {a: [] for a in arms}
        for a, (f, w) in arms.items():
            nb = w(N, O, I)
            ws = torch.empty(nb, dtype=torch.uint8, device=dev)
            dW = torch.empty(O, I, device=dev)
            db = torch.empty(O, device=dev)
            outs[a] = (f, ws, nb, dW, db)

        def run(a):
            f, ws, nb, dW, db = outs[a]
            rc = f(gy.data_ptr(), O, x.data_ptr(), I, N, O, I, dW.data_ptr(), db.data_ptr(), ws.data_ptr(), nb,
                   stream_handle(dev))
            assert rc == 0
        for a in arms:
            run(a)
        torch.cuda.synchronize()
        same = bool(torch.equal(outs["new"][3], outs["old"][3]) and torch.equal(outs["new"][4], outs["old"][4]))
        for _ in range(7):
            for a in arms:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    run(a)
                e1.record()
                torch.cuda.synchronize()
                t[a].append(e0.elapsed_time(e1) / 20 * 1e3)
        rec = dict(shape=[N, O, I], bitwise_equal=same)
        for a in arms:
            us = sorted(t[a])[3]
            tot[a] += us
            rec[a + "_us"] = round(us, 1)
            rec[a + "_tflops"] = round(2.0 * N * O * I / (us * 1e-6) / 1e12, 1)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_us": {a: round(v, 1) for a, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
