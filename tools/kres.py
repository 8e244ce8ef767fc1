#!/usr/bin/env python3
"""Per-kernel VGPRs / AGPRs / spills / LDS / occupancy of one HIP source (hipcc resource remarks):
   python3 tools/kres.py rq-vae-recommender_amd/csrc/attention.hip [name-filter] ["extra hipcc flags"]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
extra = sys.argv[3].split() if len(sys.argv) > 3 else []
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                      *extra, "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = {"name": name.split("(")[0]}
        rows.append(cur)
        continue
    for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("spill", r"VGPRs Spill: (\d+)"),
                     ("lds", r"LDS Size \[bytes/block\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None:
            cur[key] = m.group(1)
for r in rows:
    if flt in r["name"]:
        print(f"{r['name']:60s} vgpr={r.get('vgpr')} agpr={r.get('agpr')} spill={r.get('spill')} "
              f"lds={r.get('lds')} occ={r.get('occ')}")
