"""Sum rocprofv3 --pmc counters per kernel name (substring) over a counter_collection.csv tree.

usage: python tools/pmc_kernel_sum.py <dir> <kernel substring> [last N dispatches]
"""
import collections
import csv
import glob
import os
import sys

d, k = sys.argv[1], sys.argv[2]
last = int(sys.argv[3]) if len(sys.argv) > 3 else 0
rows = []
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if k in r["Kernel_Name"]]
ids = sorted({int(r["Dispatch_Id"]) for r in rows})
if last:
    keep = set(ids[-last:])
    rows = [r for r in rows if int(r["Dispatch_Id"]) in keep]
tot = collections.defaultdict(float)
for r in rows:
    tot[r["Counter_Name"]] += float(r["Counter_Value"])
n = len(ids[-last:]) if last else len(ids)
print(f"{k}: {n} dispatches")
for c, v in sorted(tot.items()):
    print(f"  {c:28s} total {v:16.0f}  per dispatch {v / max(1, n):14.1f}")
