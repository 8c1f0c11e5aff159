"""Phase timeline of k_tail (the persistent tail loop) from a -DGBPE_KTRACE build:
every 16th merge, workgroup slot 1 holds k_tail's stamps (µs from the merge's
loop start), slot 0 the zone pass's (zone_one) stamps.  Medians per merge bucket.

usage: python tools/ktrace_tail.py <dump file>
"""
import os
import sys

import numpy as np

EVERY, WG, SLOTS, HZ = 16, 2048, 12, 100e6


def main():
    raw = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 2 * WG, SLOTS)
    names = ["sel", "cand", "filt", "body", "zone", "flush", "remax", "n_remax", "ntok", "nfilt",
             "z_load", "z_sites", "z_scan", "z_keep", "z_win", "z_wrote"]
    rows = []
    for i in range(raw.shape[0]):
        tl, z = raw[i, 1].astype(np.float64), raw[i, 0].astype(np.float64)
        if tl[0] == 0 or tl[7] == 0:
            continue
        us = lambda x: (x - tl[0]) / HZ * 1e6
        rows.append([i * EVERY] + [us(tl[k]) for k in range(1, 8)] + [tl[9], tl[10], tl[11]] +
                    [us(z[k]) if z[k] else np.nan for k in (2, 3, 7, 8, 9, 4)])
    a = np.array(rows)
    edges = [int(e) for e in os.environ.get("EDGES", "0,2000,4000,8000,16000,24000,40000,60000").split(",")]
    print(f"{'merges':<13}{'n':>5}" + "".join(f"{k:>9}" for k in names))
    for lo, hi in zip(edges[:-1], edges[1:]):
        m = (a[:, 0] >= lo) & (a[:, 0] < hi)
        if m.any():
            print(f"{lo:>6}-{hi:<6}{int(m.sum()):>5}" + "".join(f"{np.nanmedian(a[m, j]):>9.2f}" for j in range(1, a.shape[1])))


if __name__ == "__main__":
    main()
