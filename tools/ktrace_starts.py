"""Workgroup start offsets of k_body (-DGBPE_KTRACE dump): for traced merges in
[lo, hi), the start of each workgroup relative to the first, by blockIdx decile.
usage: python tools/ktrace_starts.py <dump> lo hi"""
import sys
import numpy as np
EVERY, WG, SLOTS, HZ = 16, 2048, 12, 100e6
raw = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 2 * WG, SLOTS)
lo, hi = int(sys.argv[2]), int(sys.argv[3])
rows = []
for i in range(raw.shape[0]):
    if not (lo <= i * EVERY < hi):
        continue
    body = raw[i, :WG]
    on = np.flatnonzero(body[:, 0] > 0)
    if len(on) == 0:
        continue
    st = body[on, 0].astype(np.float64)
    en = body[on, 5].astype(np.float64)
    t0 = st.min()
    rows.append(((st - t0) / HZ * 1e6, (en - t0) / HZ * 1e6, on))
for name, k in (("start", 0), ("end", 1)):
    print(name)
    for q in range(10):
        vals = []
        for r in rows:
            n = len(r[2]); sel = (r[2] >= n * q // 10) & (r[2] < n * (q + 1) // 10)
            vals.append(np.median(r[k][sel]))
        print(f"  decile {q}: median {np.median(vals):7.2f} us")
allst = np.concatenate([r[0] for r in rows])
print("start percentiles", np.percentile(allst, [10, 50, 90, 99, 100]).round(2))
