"""Per-merge kernel durations of a profiled bench.py train leg, bucketed by merge
index, next to the merge counts dumped with BENCH_DUMP_MERGES.

Every kernel launch is attributed to the merge whose k_refresh (one per merge,
its last kernel) follows it, so dense merges (k_delta + k_compact) and
sector-sparse merges (k_body + zone k_delta + zone k_compact) share one table.  Only the last run of
the workload in the trace is used (the one BENCH_DUMP_MERGES dumped).

usage: [EDGES=0,10,100] python tools/merge_profile.py <rocprof csv dir> <merges.npy>
(k_sp_ = the sparse loop's entry / shrink / filter-rebuild kernels)
"""
import csv
import glob
import os
import sys

import numpy as np

KS = ["k_select", "k_body", "k_zseg", "k_delta", "k_compact", "k_refresh", "k_sp_"]


def main():
    rows = []
    for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    m = np.load(sys.argv[2])
    nm = len(m)
    refs = [i for i, r in enumerate(rows) if "k_refresh" in r["Kernel_Name"]][-nm:]
    sel = refs
    d = {k: np.zeros(nm) for k in KS}
    j = 0
    for i in range(refs[0] - 1, -1, -1):   # the first merge's other kernels, back to the previous refresh
        if "k_refresh" in rows[i]["Kernel_Name"]:
            break
        first = i
    for i in range(first, refs[-1] + 1):
        r = rows[i]
        name = r["Kernel_Name"]
        for k in KS:
            if k in name:
                d[k][j] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                break
        if "k_refresh" in name:
            j += 1
    starts = np.array([int(rows[i]["Start_Timestamp"]) for i in sel], dtype=np.float64)
    period = np.diff(starts) / 1e3
    print(f"{'merges':<14}{'count':>9}" + "".join(f"{k:>11}" for k in KS) + f"{'sum':>9}{'period':>9}")
    edges = [int(e) for e in os.environ["EDGES"].split(",")] + [nm] if os.environ.get("EDGES") else \
        [0, 100, 500, 1000, 2000, 4000, 8000, 16000, 24000, nm]
    for a, b in zip(edges[:-1], edges[1:]):
        if a >= nm:
            break
        b = min(b, nm)
        tot = sum(d[k][a:b].mean() for k in KS)
        print(f"{a:>6}-{b:<7}{int(np.median(m[a:b, 3])):>9}" + "".join(f"{d[k][a:b].mean():>11.1f}" for k in KS)
              + f"{tot:>9.1f}{period[a:max(a + 1, b - 1)].mean():>9.1f}")
    print("total ms " + " ".join(f"{k}={d[k].sum() / 1e3:.1f}" for k in KS) +
          f" span={(starts[-1] - starts[0]) / 1e6:.1f}")


if __name__ == "__main__":
    main()
