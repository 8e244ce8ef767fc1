#!/usr/bin/env python3
"""In-process A/B of rq_gemm_bf16x3_ex between the current library and another build of the same
entry point (a standalone .so of linear.hip + dropout.hip built with different macros), at the
RQ-VAE MLP launch shapes (split operands / epilogues as the fused chain issues them). Interleaved
rounds, HIP events.

  python tools/ab_gemm3.py tools/_ab_x3_mfma32.so [dec]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import torch  # noqa: E402

from rqvae_hip import _lib, ops  # noqa: E402
from rqvae_hip._lib import stream_handle  # noqa: E402

P, I64, I, F, U64, SZ = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_uint64, ctypes.c_size_t
SIG = [P, P, I64, I, P, P, I64, I, I64, I64, I64, P, I64, I, P, P, P, I64, F, U64, P, SZ, P]

# (M, N, K, a_kc, a_split, b_kc, b_split, epilogue): the fused RQ-VAE chain's launches (B = 65,536)
CASES = [(65536, 512, 768, 1, 0, 1, 1, 1), (65536, 256, 512, 1, 1, 1, 1, 1), (65536, 768, 512, 1, 1, 1, 1, 0),
         (65536, 512, 256, 1, 1, 1, 1, 1), (65536, 512, 256, 1, 1, 0, 1, 2), (65536, 512, 768, 1, 0, 0, 1, 2),
         (512, 768, 65536, 0, 0, 0, 0, 0), (768, 512, 65536, 0, 0, 0, 1, 0), (256, 512, 65536, 0, 1, 0, 1, 0),
         (65536, 128, 256, 1, 1, 1, 1, 1), (65536, 64, 128, 1, 1, 1, 1, 0)]


# decoder weight grads (rows = bucketed context / future tokens of a 256-sequence batch)
DEC_CASES = [(O, I, R, 0, 0, 0, 0, 0) for R in (12288, 20480) for (O, I) in ((512, 512), (1536, 512), (1024, 512),
                                                                             (512, 1024))]


def bind(lib):
    f = lib.rq_gemm_bf16x3_ex
    f.argtypes, f.restype = SIG, I
    w = lib.rq_gemm_bf16x3_workspace
    w.argtypes, w.restype = [I64] * 3, SZ
    return f, w


def main():
    dev = torch.device("cuda", 0)
    arms = {"new": bind(_lib.load()), "old": bind(ctypes.CDLL(os.path.abspath(sys.argv[1])))}
    tot = {a: 0.0 for a in arms}
    cases = DEC_CASES if len(sys.argv) > 2 and sys.argv[2] == "dec" else CASES
    for (M, N, K, akc, asp, bkc, bsp, epi) in cases:
        g = torch.Generator(device=dev).manual_seed(M + N + K)
        a = torch.randn((M, K) if akc else (K, M), generator=g, device=dev)
        b = torch.randn((N, K) if bkc else (K, N), generator=g, device=dev) / K ** 0.5
        A = ops.split_bf16x3(a) if asp else None
        B = ops.split_bf16x3(b) if bsp else None
        Z = torch.randn(M, N, generator=g, device=dev)
        outs = {}
        for arm, (f, w) in arms.items():
            nb = w(M, N, K) if epi == 0 else 0
            ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
            C = torch.empty(M, N, device=dev)
            Hh = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            Hl = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            outs[arm] = (f, nb, ws, C, Hh, Hl)

        def run(arm):
            f, nb, ws, C, Hh, Hl = outs[arm]
            pa, pal = (A.hi.data_ptr(), A.lo.data_ptr()) if asp else (a.data_ptr(), None)
            pb, pbl = (B.hi.data_ptr(), B.lo.data_ptr()) if bsp else (b.data_ptr(), None)
            rc = f(pa, pal, a.shape[1], akc, pb, pbl, b.shape[1], bkc, M, N, K, C.data_ptr(), N, epi,
                   Z.data_ptr(), Hh.data_ptr(), Hl.data_ptr(), N, 0.0, 0, ws.data_ptr(), nb, stream_handle(dev))
            assert rc == 0, rc
        for arm in arms:
            run(arm)
        torch.cuda.synchronize()
        key = 4 if epi == 2 else 3
        x0, x1 = (outs["new"][key].float(), outs["old"][key].float())
        rel = float((x0 - x1).abs().max() / x1.abs().max())
        t = {arm: [] for arm in arms}
        for _ in range(7):
            for arm in arms:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    run(arm)
                e1.record()
                torch.cuda.synchronize()
                t[arm].append(e0.elapsed_time(e1) / 10 * 1e3)
        rec = dict(case=[M, N, K, akc, asp, bkc, bsp, epi], rel_diff=rel)
        for arm in arms:
            us = sorted(t[arm])[3]
            tot[arm] += us
            rec[arm + "_us"] = round(us, 1)
            rec[arm + "_tflops"] = round(2.0 * M * N * K / (us * 1e-6) / 1e12, 1)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_us": {a: round(v, 1) for a, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
