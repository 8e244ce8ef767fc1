#!/usr/bin/env python3
"""Per-step device time by kernel category from a rocprofv3 kernel_stats.csv:
   python3 tools/kcat.py <kernel_stats.csv> <steps>"""
import csv
import re
import sys

CATS = [("attention", r"attn_"), ("gemm", r"gemm_bf16x3|gemm_x3w"), ("splitk_reduce", r"x3_reduce"),
        ("rmsnorm", r"rmsnorm|rms_reduce"), ("optimizer", r"adamw"), ("split", r"split_bf16x3"),
        ("dropout/silu", r"dropout|silu"), ("jagged/embedding", r"jagged|embed|segsum|gather|scatter|col_sum|batch"),
        ("torch", r"at::native|elementwise|reduce_kernel"), ("other", r".")]
rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
agg = {}
for r in rows:
    for c, pat in CATS:
        if re.search(pat, r["Name"]):
            a = agg.setdefault(c, [0.0, 0])
            a[0] += float(r["TotalDurationNs"]) / 1e3 / steps
            a[1] += int(r["Calls"]) / steps
            break
tot = sum(v[0] for v in agg.values())
for c, (us, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print(f"{c:18s} {us:9.1f} us/step {n:7.1f} launches/step {100 * us / tot:5.1f} %")
print(f"{'total':18s} {tot:9.1f} us/step {sum(v[1] for v in agg.values()):7.1f} launches/step")
