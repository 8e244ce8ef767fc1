"""Kernel-level A/B of the attention launches at the Amazon encoder shape (256 sequences, 8 heads, hd 64,
n = 4 U{2..20} + 1 tokens, non-causal self-attention) and the ML-32M shape (`--ml32m`: 64 x 6 heads, causal,
n <= 801): forward and backward timed separately with HIP events (median of 50), split-bf16 forms on / off
(matmul 'high'). One JSON line per (pass, mode)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, n=50):
    ts = []
    for _ in range(n + 5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return float(np.median(ts[5:]))


def main():
    from rqvae_hip import ops
    dev = torch.device("cuda", 0)
    torch.set_float32_matmul_precision("high")
    g = np.random.default_rng(0)
    if "--ml32m" in sys.argv:
        B, H, causal = 64, 6, True
        lens = 4 * g.integers(2, 201, B) + 1
    else:
        B, H, causal = 256, 8, False
        lens = 4 * g.integers(2, 21, B) + 1
    A = H * 64
    cu = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)).to(dev)
    T, mx = int(lens.sum()), int(lens.max())
    q, k, v, do = (torch.randn(T, A, device=dev) for _ in range(4))
    flags = [int(f) for f in os.environ.get("PROBE_FLAGS", "0").split(",")]
    modes = os.environ.get("PROBE_MODES", "x3,fp32").split(",")
    # the decoder's cross-attention at the same contexts: L+2 = 5 future queries per sequence
    nf = 5
    cuq = torch.arange(B + 1, device=dev, dtype=torch.int64) * nf
    qc, doc = torch.randn(B * nf, A, device=dev), torch.randn(B * nf, A, device=dev)
    for rnd in range(int(os.environ.get("PROBE_ROUNDS", "1"))):
        for fl in flags:
            for mode in modes:
                ops._ATTN_X3 = ops._ATTN_X3_BWD = mode == "x3"
                with ops.attn_policy(fl):
                    qs, ks, vs = (t.clone().requires_grad_(True) for t in (q, k, v))
                    fwd = timed(lambda: ops.varlen_attention(qs, ks, vs, cu, cu, H, causal, mx, mx))
                    o = ops.varlen_attention(qs, ks, vs, cu, cu, H, causal, mx, mx)
                    bwd = timed(lambda: torch.autograd.grad(o, (qs, ks, vs), do, retain_graph=True))
                    xq, xk, xv = (t.clone().requires_grad_(True) for t in (qc, k, v))
                    cf = timed(lambda: ops.varlen_attention(xq, xk, xv, cuq, cu, H, False, nf, mx))
                    oc = ops.varlen_attention(xq, xk, xv, cuq, cu, H, False, nf, mx)
                    cb = timed(lambda: torch.autograd.grad(oc, (xq, xk, xv), doc, retain_graph=True))
                print(json.dumps({"B": B, "H": H, "causal": causal, "tokens": T, "mode": mode, "flags": fl, "round": rnd,
                                  "fwd_us": round(fwd, 1), "bwd_us": round(bwd, 1), "cross_fwd_us": round(cf, 1),
                                  "cross_bwd_us": round(cb, 1)}), flush=True)
    ops._ATTN_X3 = ops._ATTN_X3_BWD = True


if __name__ == "__main__":
    main()
