#!/usr/bin/env python3
"""Same-process A/B of the RQ-VAE bench step (65,536 items, ML-32M dims): weight-grad GEMMs on the
main stream vs a side stream (ops.wgrad_stream_enable: they overlap the data-grad chain, so their
epilogue bursts and the data-grad GEMMs' stop coinciding), both with flat-bucket direct gradients.
   python3 tools/rq_side_ab.py [steps] [rounds]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from data.schemas import SeqBatch  # noqa: E402
from rqvae_hip import dp, ops  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
model = bench.build_model(dev)
buckets = dp.GradBuckets([list(model.decoder.parameters()) + list(model.layers.parameters()),
                          list(model.encoder.parameters())], flat_views=True)
opt = bench.make_adamw(model.parameters(), bench.CFG["lr"], bench.CFG["wd"])
gen = torch.Generator(device=dev).manual_seed(1000)
pool = [bench.make_items(65536, bench.CFG["input_dim"], gen, dev) for _ in range(4)]
it = [0]


def step():
    xb = pool[it[0] % 4]
    it[0] += 1
    buckets.zero_grad()
    out = model(SeqBatch(None, None, None, xb, None, None), gumbel_t=0.2)
    out.loss.backward()
    buckets.synchronize()
    opt.step()


res = {"main": [], "side": []}
for r in range(rounds):
    for mode in ("main", "side"):
        ops.wgrad_stream_enable(mode == "side")
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        res[mode].append(round((time.perf_counter() - t0) / steps * 1e3, 4))
ops.wgrad_stream_enable(False)
print(json.dumps({"ms_per_step": res, "best": {k: min(v) for k, v in res.items()}}), flush=True)
