"""Per-kernel durations and inter-kernel gaps of the last merges of a
rocprofv3 --kernel-trace CSV (sharded or single training loop).

usage: python tools/sharded_gaps.py <csv dir> [last_n_dispatches]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

import numpy as np

NAMES = ["k_select", "k_delta", "k_shard_list", "k_shard_header", "k_shard_apply", "k_compact", "k_shard_append",
         "k_refresh", "copyBuffer", "ncclDevKernel", "AllGather"]


def short(n):
    for k in NAMES:
        if k in n:
            return k
    return n[:24]


def main():
    rows = []
    for f in glob.glob(os.path.join(sys.argv[1], "*kernel_trace.csv")):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    rows = rows[-last:]
    dur, gap = defaultdict(list), defaultdict(list)
    for p, q in zip(rows[:-1], rows[1:]):
        dur[short(p["Kernel_Name"])].append((int(p["End_Timestamp"]) - int(p["Start_Timestamp"])) / 1e3)
        gap[(short(p["Kernel_Name"]), short(q["Kernel_Name"]))].append(
            (int(q["Start_Timestamp"]) - int(p["End_Timestamp"])) / 1e3)
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print(f"dur {k:<20} n={len(v):<7} mean={np.mean(v):8.2f} us")
    for k, v in sorted(gap.items(), key=lambda kv: -len(kv[1])):
        if len(v) > 50:
            print(f"gap {k[0]:>16} -> {k[1]:<16} n={len(v):<7} median={np.median(v):7.2f} mean={np.mean(v):7.2f} us")


if __name__ == "__main__":
    main()
