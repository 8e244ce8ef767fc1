#!/usr/bin/env python3
"""Per-(kernel, grid) duration summary of a rocprofv3 kernel trace, for kernels whose statistics
rocprof aggregates over several launch shapes (e.g. one GEMM instantiation used by several layers).

  python tools/trace_shapes.py gpurun_out/prof/rqvae_kernel_trace.csv [name-substring]
"""
import collections
import csv
import json
import sys


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "gemm_bf16x3"
    groups = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if sub in r["Kernel_Name"]:
            key = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))
            groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for (name, wgs), v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        print(json.dumps({"kernel": name, "workgroups": wgs, "launches": len(v), "mean_us": round(sum(v) / len(v), 2),
                          "median_us": round(v[len(v) // 2], 2)}))


if __name__ == "__main__":
    main()
