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

# per merge (a merge ends at its k_refresh): kernels numbered by repeat within the
# merge (k_delta_mt#0 = tiles, #1 = stale tail under GBPE_SPLIT_TAIL), bucketed
import os
edges = [int(x) for x in os.environ.get("EDGES", "0,10,50,128,300,1000,4000,16000,1073741824").split(",")]
merges, curm, spans = [], [], []
mstart = None
for r in rows:
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].replace("void ", "")
    s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if mstart is None:
        mstart = s0
    curm.append((k, (e0 - s0) / 1e3))
    if k == "k_refresh":
        merges.append(curm)
        spans.append((e0 - mstart) / 1e3)
        curm, mstart = [], e0
print(f"--- per merge ({len(merges)} k_refresh-terminated groups; group 0 holds the creation / entry kernels)")
for a, b in zip(edges[:-1], edges[1:]):
    sel = merges[a:b]
    if not sel:
        break
    acc = defaultdict(float)
    for m in sel:
        seen = defaultdict(int)
        for k, us in m:
            acc[f"{k}#{seen[k]}"] += us
            seen[k] += 1
    tot = sum(acc.values())
    span = sum(spans[a:b]) / len(sel)
    print(f"merges {a}-{a + len(sel)}: {tot / len(sel):8.1f} us busy, {span:8.1f} us span /merge  " +
          "  ".join(f"{k} {v / len(sel):.1f}" for k, v in sorted(acc.items(), key=lambda kv: -kv[1])[:9]))
