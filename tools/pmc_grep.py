"""Print the counters of the dispatches whose kernel name contains a pattern
(rocprofv3 --pmc CSV output; kernel names contain commas, so parse as CSV).

usage: python tools/pmc_grep.py <dir> <pattern> [--delete]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d, pat = sys.argv[1], sys.argv[2]
    agg = defaultdict(list)
    files = glob.glob(os.path.join(d, "*counter_collection.csv"))
    for f in files:
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(f"{k}: n={len(v)} mean={sum(v) / len(v):.4g} last={v[-1]:.4g}")
    if "--delete" in sys.argv:
        for f in files:
            os.remove(f)


if __name__ == "__main__":
    main()
