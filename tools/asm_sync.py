#!/usr/bin/env python3
"""Synchronisation skeleton of one kernel in a hipcc --save-temps .s file: the waitcnt / barrier /
setprio / branch lines (with the count of MFMA, LDS-read and LDS-DMA instructions between them),
to check that a pipelined loop has no compiler-inserted vmcnt(0) and its waits sit where intended.
   python3 tools/asm_sync.py file.s kernel_substring [max_lines]"""
import re
import sys

path, key = sys.argv[1], sys.argv[2]
limit = int(sys.argv[3]) if len(sys.argv) > 3 else 400
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if re.match(r"^\S+:", l) and key in l.split(":")[0])
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = [l.strip() for l in lines[start:end]]
totals, run, out = {}, {}, []
kinds = {"v_mfma": "mfma", "ds_read": "dsr", "ds_write": "dsw", "global_load_lds": "glds", "global_load": "gld",
         "global_store": "gst", "scratch_": "scratch"}
for l in body:
    op = l.split()[0] if l else ""
    k = next((v for p, v in kinds.items() if op.startswith(p)), None)
    if k:
        totals[k] = totals.get(k, 0) + 1
        run[k] = run.get(k, 0) + 1
        continue
    if op.startswith(("s_waitcnt", "s_barrier", "s_setprio", "s_cbranch", "s_branch")) or l.startswith(".LBB"):
        if run:
            out.append("    " + " ".join(f"{a}={b}" for a, b in run.items()))
            run = {}
        out.append(l)
print("totals:", totals)
print("\n".join(out[:limit]))
