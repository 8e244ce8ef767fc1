#!/usr/bin/env python3
"""Busy vs idle time of the GPU between consecutive AdamW launches (one train step each) in a
rocprofv3 kernel trace, plus the per-step kernel count and the largest idle gaps' neighbours.
   python tools/step_gaps.py gpurun_out/prof/decoder_kernel_trace.csv [adamw_substring]"""
import csv
import sys

path = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else "adamw_kernel"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:90]) for r in rows]
marks = [i for i, k in enumerate(ks) if key in k[2]]
steps = []
for a, b in zip(marks, marks[1:]):
    seg = ks[a + 1:b + 1]
    wall = seg[-1][1] - ks[a][1]
    busy, end = 0, ks[a][1]
    gaps = []
    for s, e, n in seg:
        if s > end:
            gaps.append((s - end, n))
        busy += max(0, e - max(s, end))
        end = max(end, e)
    steps.append((wall, busy, len(seg), gaps))
steps = steps[-12:]
for wall, busy, n, gaps in steps:
    print(f"step wall {wall/1e3:8.1f} us busy {busy/1e3:8.1f} us idle {100*(1-busy/wall):5.1f}% kernels {n}")
wall, busy, n, gaps = steps[-1]
gaps.sort(reverse=True)
tot = sum(g for g, _ in gaps)
print(f"last step: {len(gaps)} gaps, {tot/1e3:.1f} us; largest:")
for g, nm in gaps[:12]:
    print(f"  {g/1e3:7.1f} us before {nm}")
