"""Per-merge kernel durations of a profiled bench.py train leg, bucketed by merge
index, next to the merge counts dumped with BENCH_DUMP_MERGES.

usage: python tools/merge_profile.py <rocprof csv dir> <merges.npy>
"""
import csv
import glob
import os
import sys

import numpy as np


def main():
    rows = []
    for f in glob.glob(os.path.join(sys.argv[1], "*kernel_trace.csv")):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    m = np.load(sys.argv[2])
    nm = len(m)

    def ser(k, field=None):
        return np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) if field is None
                         else int(r[field]) for r in rows if k in r["Kernel_Name"]], dtype=np.float64)[-nm:]

    ks = ["k_select", "k_delta", "k_compact", "k_refresh"]
    d = {k: ser(k) / 1e3 for k in ks}
    starts = ser("k_select", "Start_Timestamp")
    period = np.diff(starts) / 1e3
    print(f"{'merges':<14}{'count':>9}" + "".join(f"{k:>11}" for k in ks) + f"{'sum':>9}{'period':>9}")
    edges = [0, 100, 500, 1000, 2000, 4000, 8000, 16000, 24000, nm]
    for a, b in zip(edges[:-1], edges[1:]):
        if a >= nm:
            break
        b = min(b, nm)
        tot = sum(d[k][a:b].mean() for k in ks)
        print(f"{a:>6}-{b:<7}{int(np.median(m[a:b, 3])):>9}" + "".join(f"{d[k][a:b].mean():>11.1f}" for k in ks)
              + f"{tot:>9.1f}{period[a:b - 1].mean():>9.1f}")
    print("total ms " + " ".join(f"{k}={d[k].sum() / 1e3:.1f}" for k in ks) +
          f" span={(starts[-1] - starts[0]) / 1e6:.1f}")


if __name__ == "__main__":
    main()
