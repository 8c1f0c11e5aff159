"""Idle gaps between consecutive kernels of a rocprofv3 --kernel-trace run
(diagnostic): for the k_body / k_refresh pairs of the sparse loop, the gap
before each kernel, split into within-step and step-boundary gaps, over merge
windows.  usage: python tools/trace_gaps.py <trace dir>"""
import csv
import glob
import os
import sys

import numpy as np

rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name = [r["Kernel_Name"] for r in rows]
st = np.array([int(r["Start_Timestamp"]) for r in rows], dtype=np.int64)
en = np.array([int(r["End_Timestamp"]) for r in rows], dtype=np.int64)
gap = np.zeros(len(rows))
gap[1:] = (st[1:] - en[:-1]) / 1e3
dur = (en - st) / 1e3
isb = np.array(["k_body" in n for n in name])
isr = np.array(["k_refresh" in n for n in name])
bi = np.flatnonzero(isb)
print(f"kernels {len(rows)}, k_body {len(bi)}, k_refresh {isr.sum()}, span {(en[-1] - st[0]) / 1e6:.1f} ms, "
      f"busy {dur.sum() / 1e3:.1f} ms, idle {gap[gap > 0].sum() / 1e3:.1f} ms")
print("merges        k_body_us  gap_before_body  refresh_us  gap_before_refresh  other_kernels_between  step_gaps>20us")
for lo, hi in [(0, 512), (512, 4096), (4096, 8192), (8192, 16384), (16384, 24576), (24576, len(bi))]:
    sel = bi[lo:hi]
    if not len(sel):
        continue
    nxt = sel + 1
    nxt = nxt[nxt < len(rows)]
    ref = nxt[isr[nxt]]
    other = 0
    gb = gap[sel]
    print(f"{lo:6d}-{hi:6d}  {np.median(dur[sel]):9.2f}  {np.median(gb):15.2f}  {np.median(dur[ref]) if len(ref) else float('nan'):10.2f}"
          f"  {np.median(gap[ref]) if len(ref) else float('nan'):18.2f}  {len(nxt) - len(ref):21d}  {int((gb > 20).sum()):6d}"
          f"  (mean gap before body {gb.mean():.2f}, sum {gb.sum() / 1e3:.2f} ms)")
