"""Kernel timeline of a rocprofv3 --kernel-trace run (diagnostic): per kernel
name, launches / total / mean µs, then the first N launches in order with the
gap before each (idle device time).  usage: python tools/trace_timeline.py <dir> [N]"""
import csv
import glob
import os
import sys
from collections import defaultdict

rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
N = int(sys.argv[2]) if len(sys.argv) > 2 else 200
agg = defaultdict(lambda: [0, 0.0])
for r in rows:
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3 if rows else 0
print(f"kernels {len(rows)}  busy {tot / 1e3:.2f} ms  span {span / 1e3:.2f} ms")
for k, (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{us / 1e3:10.3f} ms {c:8d} x {us / c:9.2f} us  {k[-90:]}")
print("--- first launches: start(us) dur(us) gap(us) grid name")
t0 = int(rows[0]["Start_Timestamp"]) if rows else 0
prev_end = t0
for r in rows[:N]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = r.get("Grid_Size_X", r.get("Grid_Size", ""))
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-70:]
    print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f} {(s - prev_end) / 1e3:8.1f} {g:>9} {name}")
    prev_end = max(prev_end, e)
