#!/usr/bin/env python3
"""Late-merge kernel timeline from a rocprofv3 --kernel-trace CSV (diagnostic):
for the last N k_body dispatches, the median k_body and k_refresh durations, the
k_body -> k_refresh gap, the k_refresh -> next k_body gap and the period.

    python tools/ktrace_late.py <kernel_trace.csv> [N]
"""
import csv
import sys

import numpy as np


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
    body = [i for i, r in enumerate(rows) if "k_body" in r[2]]
    sel = body[-n:]
    d_body, d_ref, g1, g2, per = [], [], [], [], []
    for j, i in enumerate(sel):
        s, e, _ = rows[i]
        d_body.append(e - s)
        if i + 1 < len(rows) and "k_refresh" in rows[i + 1][2]:
            rs, re_, _ = rows[i + 1]
            d_ref.append(re_ - rs)
            g1.append(rs - e)
            if i + 2 < len(rows) and "k_body" in rows[i + 2][2]:
                g2.append(rows[i + 2][0] - re_)
                per.append(rows[i + 2][0] - s)
    med = lambda v: float(np.median(v)) / 1e3 if v else float("nan")
    print("last %d k_body (%s): k_body %.2f us, gap %.2f, k_refresh %.2f, gap %.2f, period %.2f (medians, us)"
          % (len(sel), rows[sel[0]][2][:60], med(d_body), med(g1), med(d_ref), med(g2), med(per)))
    for q in (10, 50, 90):
        print("  p%d k_body %.2f k_refresh %.2f period %.2f" % (q, np.percentile(d_body, q) / 1e3,
                                                             np.percentile(d_ref, q) / 1e3 if d_ref else 0,
                                                             np.percentile(per, q) / 1e3 if per else 0))


if __name__ == "__main__":
    main()
