#!/usr/bin/env python3
"""Summary of tools/ab_lib.sh output: per-shape x3 / x3s / auto us (A = tree build, B = other) and
the bench steps.   python tools/ab_lib_summary.py [tag]"""
import glob
import json
import sys

T = sys.argv[1] if len(sys.argv) > 1 else "ab"
O = "gpurun_out/ablib"
A = [json.loads(l) for l in open(f"{O}/{T}_shapes_A.jsonl")]
B = [json.loads(l) for l in open(f"{O}/{T}_shapes_B.jsonl")]
for a, b in zip(A, B):
    print(f"{a['shape']:22s} x3 {b['x3']:6.1f} -> {a['x3']:6.1f}  x3s {b['x3s']:6.1f} -> {a['x3s']:6.1f}  "
          f"auto {b['auto']:6.1f} -> {a['auto']:6.1f} {a['auto_plan']}")


def line(f):
    for l in open(f):
        if l.startswith("{"):
            return json.loads(l)


for f in sorted(glob.glob(f"{O}/{T}_bench_*.json")):
    d = line(f)
    print(f.split("/")[-1], "rqvae", d["ms_per_step"], "decoder", d.get("decoder_amazon", {}).get("ms_per_step"),
          "gemm frac", d["roofline"]["frac"])
