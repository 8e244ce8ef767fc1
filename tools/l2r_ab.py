"""A/B of the l2norm + reconstruction kernels' rows per wave (1 / 2 / 4) at the RQ-VAE ML-32M head
shape (B = 65,536, C = 768): average fwd and split-bwd launch time, HIP events on the launch stream."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rq-vae-recommender_amd"))
from rqvae_hip import _lib  # noqa: E402
from rqvae_hip._lib import call, ptr, stream_handle  # noqa: E402


def main(B=65536, C=768, iters=200):
    dev = torch.device("cuda:0")
    pre = torch.randn(B, C, device=dev)
    x = torch.nn.functional.normalize(torch.randn(B, C, device=dev), dim=-1)
    rec = torch.empty(B, device=dev)
    nrm = torch.empty(B, device=dev)
    gr = torch.rand(B, device=dev)
    hi = torch.empty(B, C, device=dev, dtype=torch.int16)
    lo = torch.empty_like(hi)
    s = stream_handle(dev)
    lib = _lib.load()
    byt_f, byt_b = 2 * B * C * 4, 3 * B * C * 4
    for rep in range(2):
        for rpw in (1, 2, 4):
            lib.rq_l2norm_recon_rows_per_wave(rpw)
            res = []
            for name, args, byt in (("fwd", ("rq_l2norm_recon_fwd", ptr(pre), ptr(x), B, C, ptr(rec), ptr(nrm), s), byt_f),
                                    ("bwd_split", ("rq_l2norm_recon_bwd_split", ptr(pre), ptr(x), ptr(nrm), ptr(gr), B, C,
                                                   ptr(hi), ptr(lo), s), byt_b)):
                for _ in range(10):
                    call(*args)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(iters):
                    call(*args)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / iters
                res.append(f"{name} {us:.1f} us {byt / us / 1e3:.0f} GB/s")
            print(rep, "rpw", rpw, " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
