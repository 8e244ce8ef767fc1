#!/usr/bin/env python3
"""Summarise rocprofv3 SQ counter passes (counter_collection.csv files of the same program, one pass
each) per kernel: mean counter values over the kernel's dispatches, and the ratios used in DESIGN
(VALU : MFMA instructions, wait share of wave cycles, LDS bank-conflict cycles per LDS instruction,
MFMA busy share of the SIMD cycles = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs),
approximate: the two counters come from different runs of the same program).

  python tools/pmc_summary.py <tag> <csv> [<csv> ...]
"""
import collections
import csv
import sys


def main():
    tag, paths = sys.argv[1], sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    grid = {}
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rqhip::", "")
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            grid[k] = r["Grid_Size"]
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        out = {"tag": tag, "kernel": k[:110], "grid": grid[k], "dispatches": max(len(v) for v in cs.values())}
        out.update({c: round(v) for c, v in sorted(m.items())})
        if m.get("SQ_INSTS_MFMA"):
            out["valu_per_mfma"] = round(m.get("SQ_INSTS_VALU", 0) / m["SQ_INSTS_MFMA"], 2)
        if m.get("SQ_WAVE_CYCLES"):
            out["wait_any_frac"] = round(m.get("SQ_WAIT_ANY", 0) / m["SQ_WAVE_CYCLES"], 3)
            out["wait_inst_any_frac"] = round(m.get("SQ_WAIT_INST_ANY", 0) / m["SQ_WAVE_CYCLES"], 3)
        if m.get("SQ_INSTS_LDS"):
            out["lds_conflict_cycles_per_lds_inst"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_INSTS_LDS"], 3)
        if m.get("GRBM_GUI_ACTIVE") and m.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            out["mfma_busy_frac"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024), 3)
        print(out)


if __name__ == "__main__":
    main()
