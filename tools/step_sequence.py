"""The launch sequence of ONE train step from a rocprofv3 kernel_trace.csv (steps delimited by the adamw
kernel, as tools/step_breakdown.py): index, device us, gap to the previous launch's end, kernel, grid.
  python tools/step_sequence.py <trace.csv> [step_index]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
ad = [i for i, r in enumerate(rows) if 'adamw' in r['Kernel_Name']]
segs = [(ad[j - 1] + 1, ad[j] + 1) for j in range(1, len(ad)) if ad[j] - ad[j - 1] > 5]
si = int(sys.argv[2]) if len(sys.argv) > 2 else len(segs) // 2
a, b = segs[si]
prev_end = None
for i, r in enumerate(rows[a:b]):
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('rqhip::', '')
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    prev_end = e
    print(f"{i:4d} {(e - s) / 1e3:7.1f} {gap:6.1f}  {k[:110]} g={r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}")
