"""Device-time breakdown of ONE train step from a rocprofv3 kernel_trace.csv, steps delimited by the
adamw kernel: python tools/step_breakdown.py <trace.csv> [step_index] [top]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
ad = [i for i, r in enumerate(rows) if 'adamw' in r['Kernel_Name']]
segs = [(ad[j - 1] + 1, ad[j] + 1) for j in range(1, len(ad)) if ad[j] - ad[j - 1] > 5]
si = int(sys.argv[2]) if len(sys.argv) > 2 else len(segs) // 2
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
a, b = segs[si]
seg = rows[a:b]
per = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('rqhip::', '')
    k += f" g={r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
    per[k][0] += 1
    per[k][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
busy = sum(v[1] for v in per.values())
wall = (int(seg[-1]['End_Timestamp']) - int(seg[0]['Start_Timestamp'])) / 1e3
print(f"step {si}/{len(segs)}: {len(seg)} kernels, busy {busy:.1f} us, wall {wall:.1f} us")
for k, (n, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{t:9.1f}us {t / busy * 100:5.1f}% {n:4d}x {t / n:7.1f}us  {k[:120]}")
