#!/usr/bin/env python3
"""In-process A/B of a decoder model switch on the bench's graphed decoder step (bench.measure_decoder,
fresh model + graphs per arm, interleaved rounds), at the Amazon config and ML-32M at 8 sequences:
   python3 tools/ab_hoist.py [hoist|fuse_acc] [rounds]
hoist: the decoder layers' cross-attention K/V projections as one hoisted GEMM vs one per layer."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rq-vae-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from modules.transformer import model as tm  # noqa: E402
from rqvae_hip import gemm_tuning  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "hoist"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dev = torch.device("cuda", 0)
gemm_tuning.enable()
if what != "hoist":
    raise SystemExit(what)
arms = {"off": False, "on": True}
res = {}
for r in range(rounds):
    for cfg, B in ((bench.DEC, None), (bench.DEC_DM, 8)):
        for a, v in arms.items():
            tm._HOIST_KV = v
            d = bench.measure_decoder(dev, 1, 0, cfg, B=B, steps=20, warmup=5, graphs=True, stats=False)
            res.setdefault(f"{cfg['name']}{B or ''}:{a}", []).append(d["ms_per_step"])
            print(json.dumps({"round": r, "cfg": cfg["name"], "B": B, "arm": a, "ms": d["ms_per_step"]}), flush=True)
print(json.dumps({k: min(v) for k, v in res.items()}), flush=True)
