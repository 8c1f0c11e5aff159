"""Per-phase durations of the late-merge loop k_late from a -DGBPE_KTRACE build
(csrc/late.h stamps, workgroup slot KT_WG - 1): every 16th merge, µs per phase,
medians over merge buckets.

  sel     selection over the hot set (merge start -> selection done)
  p1      zone reads and destroyed pairs; bitmap rows, candidates' extents and
          signatures in flight meanwhile; the sector list
  p2      zone writes, window pairs, sector merges
  walk    touched delta slots -> log, hot set, bound
  close   merge bookkeeping
  total   merge start -> merge closed;  ncand / nfilt  candidates, after the filter

usage: python tools/ktrace_late.py <dump file>
"""
import os
import sys

import numpy as np

EVERY, WG, SLOTS, HZ = 16, 2048, 12, 100e6


def main():
    raw = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 2 * WG, SLOTS)
    lk = raw[:, WG - 1, :].astype(np.float64)
    rows = []
    for i in range(lk.shape[0]):
        v = lk[i]
        if v[0] <= 0 or v[5] <= 0:
            continue
        d = np.diff(v[:6]) / HZ * 1e6
        rows.append([i * EVERY, *d, (v[5] - v[0]) / HZ * 1e6, int(raw[i, WG - 1, 6]) >> 16,
                     int(raw[i, WG - 1, 6]) & 0xFFFF])
    if not rows:
        print("no k_late stamps")
        return
    a = np.array(rows)
    names = ["sel", "p1", "p2", "walk", "close", "total", "ncand", "nfilt"]
    edges = [int(e) for e in os.environ.get("EDGES", "0,2000,4000,8000,12000,16000,24000,32000,50000,66000").split(",")]
    print(f"{'merges':<13}{'n':>5}" + "".join(f"{k:>9}" for k in names))
    for lo, hi in zip(edges[:-1], edges[1:]):
        sel = (a[:, 0] >= lo) & (a[:, 0] < hi)
        if sel.any():
            med = np.median(a[sel, 1:], axis=0)
            print(f"{lo:>6}-{hi:<6}{int(sel.sum()):>5}" + "".join(f"{x:9.2f}" for x in med))


if __name__ == "__main__":
    main()
