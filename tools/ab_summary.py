#!/usr/bin/env python3
"""Summarise tools/attn_ab.sh output: mean kernel time per (variant, kernel) over the repeats."""
import csv
import glob
import os
import sys
from collections import defaultdict

root, variants = sys.argv[1], sys.argv[2:]
tab = defaultdict(lambda: defaultdict(list))
for v in variants:
    for f in glob.glob(os.path.join(root, f"{v}.*", "p_kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            if "attn" in r["Name"]:
                k = r["Name"].split("(")[0].replace("void rqhip::", "")
                tab[k][v].append(float(r["TotalDurationNs"]) / int(r["Calls"]) / 1000.0)
for k in sorted(tab):
    print(f"{k:36s} " + " ".join(f"{v}={sum(tab[k][v]) / max(1, len(tab[k][v])):8.1f}us" for v in variants))
