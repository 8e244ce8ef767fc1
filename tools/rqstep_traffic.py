"""Summarise tools/rqstep_traffic.sh: per kernel (name, grid) per step — launches, device time, HBM bytes
(FETCH_SIZE x2 + WRITE_SIZE, KiB counters; MI355X_MICROARCH.md 'HBM') and the achieved rate."""
import collections
import csv
import glob
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("rqhip::", "").replace("void ", "")
    return name[:70]


def main(root, n):
    n = int(n)
    dur = collections.defaultdict(float)
    calls = collections.Counter()
    for p in glob.glob(f"{root}/trace/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            calls[k] += 1
    byts = collections.defaultdict(float)
    for sub, ctr, mul in (("fetch", "FETCH_SIZE", 2.0), ("write", "WRITE_SIZE", 1.0)):
        for p in glob.glob(f"{root}/{sub}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(p)):
                if r["Counter_Name"] == ctr:
                    byts[short(r["Kernel_Name"])] += float(r["Counter_Value"]) * 1024 * mul
    tot_us = sum(dur.values()) / n
    tot_b = sum(byts.values()) / n
    print(f"per step: {tot_us:.1f} us kernel time, {tot_b / 1e6:.1f} MB HBM ({tot_b / tot_us / 1e3:.0f} GB/s over kernel time)")
    print(f"{'us/step':>8} {'n':>3} {'MB/step':>8} {'GB/s':>6}  kernel")
    for k in sorted(dur, key=lambda k: -dur[k]):
        us, b = dur[k] / n, byts.get(k, 0.0) / n
        print(f"{us:8.1f} {calls[k] / n:3.0f} {b / 1e6:8.1f} {b / us / 1e3 if us else 0:6.0f}  {k}")


if __name__ == "__main__":
    main(*sys.argv[1:])
