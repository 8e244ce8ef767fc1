#!/usr/bin/env python3
"""Kernel-level A/B timing in ONE process (guide §5.4 rule 24): interleaved rounds, HIP events.

  python tools/bench_kernels.py [--rounds 5]

Times rq_quantize_fwd with an explicit impl (1 = LDS-tiled, 2 = register-resident) at the BASELINE quantize
shapes, the backward (rows + codebook reduction), jagged gather/scatter and varlen attention.
Prints one JSON object per measurement.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402

from rqvae_hip import ops  # noqa: E402
from rqvae_hip._lib import call, ptr, stream_handle  # noqa: E402


def ev_time(fn, iters=20):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def quantize_case(B, D, K, L, dev):
    g = torch.Generator(device=dev).manual_seed(B + D)
    x = torch.randn(B, D, generator=g, device=dev) / D ** 0.5
    cbs = torch.randn(L, K, D, generator=g, device=dev) / D ** 0.5
    csq = (cbs * cbs).sum(-1).contiguous()
    outs = dict(ids=torch.empty(B, L, dtype=torch.int64, device=dev), emb=torch.empty(L, B, D, device=dev),
                res=torch.empty(L, B, D, device=dev), ql=torch.empty(B, device=dev), es=torch.empty(B, D, device=dev))
    return x, cbs, csq, outs


def run_impl(x, cbs, csq, o, impl, mode=3):
    B, D = x.shape
    L, K, _ = cbs.shape
    call("rq_quantize_fwd", ptr(x), B, D, ptr(cbs), ptr(csq), K, L, mode, 0.25, ptr(o["ids"]), ptr(o["emb"]),
         ptr(o["res"]), ptr(o["ql"]), ptr(o["es"]), None, impl, stream_handle())


def wgrad_bench(dev, rounds):
    """dW = g^T x over N rows for every Linear of the RQ-VAE encoder / decoder (768-512-256-128-64)."""
    dims = [768, 512, 256, 128, 64]
    cases = [(65536, o, i) for i, o in zip(dims[:-1], dims[1:])] + [(65536, i, o) for i, o in zip(dims[:-1], dims[1:])]
    cases += [(262144, 512, 768)]
    for (N, O, I) in cases:
        g = torch.Generator(device=dev).manual_seed(N + O + I)
        gy = torch.randn(N, O, generator=g, device=dev)
        x = torch.randn(N, I, generator=g, device=dev)
        ref = gy.t() @ x
        dW, db = ops.linear_wgrad(gy, x, True)
        err = float((dW - ref).abs().max() / ref.abs().max())
        arms = {"hip": lambda: ops.linear_wgrad(gy, x, True), "lib": lambda: (gy.t() @ x, gy.sum(0))}
        t = {a: [] for a in arms}
        for _ in range(rounds):
            for a, fn in arms.items():
                t[a].append(ev_time(fn, 10))
        for a in arms:
            ms = sorted(t[a])[rounds // 2]
            print(json.dumps(dict(kernel="wgrad", arm=a, shape=[N, O, I], median_ms=ms,
                                  tflops=2.0 * N * O * I / (ms * 1e-3) / 1e12, rel_err=err)), flush=True)
        del gy, x, ref
        torch.cuda.empty_cache()


def gemm3_bench(dev, rounds):
    """Forward / data-grad / weight-grad of every RQ-VAE MLP layer (B = 65,536): split-bf16 GEMM
    (rq_gemm_bf16x3, precision 'high') vs the fp32 library GEMM ('highest')."""
    dims = [768, 512, 256, 128, 64]
    layers = [(i, o) for i, o in zip(dims[:-1], dims[1:])] + [(o, i) for i, o in zip(dims[:-1], dims[1:])]
    N = 65536
    tot = {"x3": 0.0, "lib": 0.0}
    for (I, O) in layers:
        g = torch.Generator(device=dev).manual_seed(I * O)
        x = torch.randn(N, I, generator=g, device=dev)
        W = torch.randn(O, I, generator=g, device=dev) / I ** 0.5
        gy = torch.randn(N, O, generator=g, device=dev)
        cases = {"fwd": (lambda: ops.linear_fwd_high(x, W), lambda: x @ W.t(), 2.0 * N * I * O),
                 "dgrad": (lambda: ops.linear_dgrad_high(gy, W), lambda: gy @ W, 2.0 * N * I * O),
                 "wgrad": (lambda: ops.linear_wgrad_high(gy, x), lambda: gy.t() @ x, 2.0 * N * I * O)}
        for name, (f3, fl, flops) in cases.items():
            r3, rl = f3(), fl()
            rel = float((r3 - rl).abs().max() / rl.abs().max())
            t = {"x3": [], "lib": []}
            for _ in range(rounds):
                t["x3"].append(ev_time(f3, 10))
                t["lib"].append(ev_time(fl, 10))
            rec = dict(kernel="gemm3", op=name, layer=[I, O], rows=N, rel_err_vs_fp32=rel)
            for a in t:
                ms = sorted(t[a])[rounds // 2]
                tot[a] += ms
                rec[a + "_ms"] = round(ms, 4)
                rec[a + "_tflops"] = round(flops / (ms * 1e-3) / 1e12, 1)
            print(json.dumps(rec), flush=True)
        del x, W, gy
        torch.cuda.empty_cache()
    print(json.dumps({"gemm3_total_ms": {a: round(v, 3) for a, v in tot.items()}}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--sweep", action="store_true", help="mode / level sweep of the ML-32M shape only")
    ap.add_argument("--wgrad", action="store_true", help="weight-grad kernel vs library g^T x at the RQ-VAE shapes")
    ap.add_argument("--gemm3", action="store_true", help="split-bf16 GEMM vs fp32 library at the RQ-VAE MLP shapes")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    results = []
    if args.wgrad:
        wgrad_bench(dev, args.rounds)
        return
    if args.gemm3:
        gemm3_bench(dev, args.rounds)
        return
    if args.sweep:
        for (B, D, K, L) in [(65536, 64, 256, 3), (65536, 64, 256, 1), (65536, 64, 256, 6)]:
            x, cbs, csq, o = quantize_case(B, D, K, L, dev)
            for impl in (1, 2):
                for mode in (0, 2, 3):
                    ms = sorted(ev_time(lambda: run_impl(x, cbs, csq, o, impl, mode), 10) for _ in range(args.rounds))
                    med = ms[len(ms) // 2]
                    print(json.dumps(dict(kernel="rq_quantize_fwd", impl=impl, mode=mode, shape=[B, D, K, L],
                                          median_ms=med, tflops=2.0 * K * D * L * B / (med * 1e-3) / 1e12)), flush=True)
        return
    shapes = [(65536, 64, 256, 3), (65536, 32, 256, 3), (262144, 64, 256, 3), (64, 64, 256, 3),
              (16384, 1024, 2048, 4), (65536, 1024, 2048, 4), (65536, 256, 1024, 3)]
    for (B, D, K, L) in shapes:
        x, cbs, csq, o = quantize_case(B, D, K, L, dev)
        impls = ([1, 2, 4] if D == 64 and K <= 288 else [1, 2]) if D <= 64 else [1, 3]
        ref = None
        for impl in impls:
            run_impl(x, cbs, csq, o, impl)
            ids = o["ids"].clone()
            if ref is None:
                ref = ids
            else:
                results.append(dict(check="ids_equal_impl1_vs_%d" % impl, shape=[B, D, K, L],
                                    frac_equal=float((ids == ref).all(1).float().mean())))
        times = {i: [] for i in impls}
        for _ in range(args.rounds):
            for impl in impls:
                times[impl].append(ev_time(lambda: run_impl(x, cbs, csq, o, impl), 10))
        flops = 2.0 * K * D * L * B
        for impl in impls:
            ms = sorted(times[impl])
            results.append(dict(kernel="rq_quantize_fwd", impl=impl, shape=[B, D, K, L], median_ms=ms[len(ms) // 2],
                                min_ms=ms[0], tflops=flops / (ms[len(ms) // 2] * 1e-3) / 1e12))
        # backward
        xr = x.clone().requires_grad_(True)
        cr = cbs.clone().requires_grad_(True)
        emb, res, ids, ql, es = ops.rq_quantize(xr, cr, ops.MODE_ROTATION, 0.25)
        ges, gq = torch.randn_like(es), torch.rand_like(ql)
        nbytes = ops._lib.load().rq_quantize_bwd_workspace(B, D, K, L)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        gx, gcb = torch.empty_like(x), torch.empty_like(cbs)

        def bwd():
            call("rq_quantize_bwd", ptr(res), ptr(ids), ptr(cbs), B, D, K, L, 3, 0.25, None, ptr(ges), None, ptr(gq),
                 ptr(gx), ptr(gcb), ptr(ws), nbytes, stream_handle())
        ms = sorted(ev_time(bwd, 10) for _ in range(args.rounds))
        results.append(dict(kernel="rq_quantize_bwd", shape=[B, D, K, L], median_ms=ms[len(ms) // 2]))
        del x, cbs, csq, o, xr, cr, emb, res, ws
        torch.cuda.empty_cache()
    for r in results:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
