#!/usr/bin/env python3
"""Probe: capture the B=64 RQ-VAE train step in a hipGraph (faulthandler on)."""
import faulthandler
import os
import sys
import time

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from data.schemas import SeqBatch  # noqa: E402
from rqvae_hip.graph import CapturedStep  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev)
    xs = bench.make_items(64, 768, torch.Generator(device=dev).manual_seed(0), dev)
    stage = sys.argv[1] if len(sys.argv) > 1 else "full"
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01, foreach=True, capturable=True)

    def fwd_only():
        with torch.no_grad():
            return model(SeqBatch(None, None, None, xs, None, None), gumbel_t=0.2).loss

    def step():
        opt.zero_grad(set_to_none=False)
        o = model(SeqBatch(None, None, None, xs, None, None), gumbel_t=0.2)
        o.loss.backward()
        opt.step()
        return o.loss.detach()
    fn = fwd_only if stage == "fwd" else step
    print("capturing", stage, flush=True)
    g = CapturedStep(fn)
    print("captured", flush=True)
    for _ in range(3):
        g()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        g()
    torch.cuda.synchronize()
    print(stage, "replay ms", (time.perf_counter() - t0) / 100 * 1e3, "loss", float(g.out), flush=True)


if __name__ == "__main__":
    main()
