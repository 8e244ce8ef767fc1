#!/usr/bin/env python3
"""Share of device time per kernel family from a rocprofv3 *_kernel_stats.csv, scaled to a step time:
   python3 tools/kstat_share.py stats.csv ms_per_step [top]"""
import csv
import re
import sys
from collections import defaultdict


def family(name):
    n = name.split("(")[0].replace("void ", "")
    n = re.sub(r"^rqhip::", "", n)
    if "at::native" in n:
        m = re.search(r"at::native::[\w:]*?(\w+_kernel\w*|\w+Functor\w*|\w+)", name)
        return "torch:" + (m.group(1) if m else n[:40])
    return n[:70]


rows = list(csv.DictReader(open(sys.argv[1])))
ms = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
tot = defaultdict(float)
calls = defaultdict(int)
for r in rows:
    f = family(r["Name"])
    tot[f] += float(r["TotalDurationNs"])
    calls[f] += int(r["Calls"])
T = sum(tot.values())
print(f"{'kernel':72s} {'share':>6s} {'ms/step':>8s} {'calls':>7s} {'us/call':>8s}")
for f, t in sorted(tot.items(), key=lambda kv: -kv[1])[:top]:
    print(f"{f:72s} {t / T:6.3f} {ms * t / T:8.3f} {calls[f]:7d} {t / calls[f] / 1e3:8.1f}")
