#!/usr/bin/env python3
"""HBM-scale jagged conversion throughput (bench.measure_jagged_c5), optionally on an A/B library build.
   python3 tools/jagged_probe.py [lib.so]"""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "rq-vae-recommender_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from rqvae_hip import _lib  # noqa: E402

if len(sys.argv) > 1:
    _lib._lib = _lib.load(sys.argv[1])
dev = torch.device("cuda", 0)
for _ in range(2):
    print(json.dumps({"lib": sys.argv[1] if len(sys.argv) > 1 else "tree", **bench.measure_jagged_c5(dev)}), flush=True)
