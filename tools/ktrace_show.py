"""Per-phase timeline of the sector-sparse kernels from a -DGBPE_KTRACE build
(tools/ktrace.sh): every 16th merge, each workgroup's wall-clock stamps (100 MHz).
Times in µs from the first k_body workgroup start; medians over merge buckets.

  start_max  last k_body workgroup to start      sel     last to finish selection
  zone       zone workgroup end                  hit_*   workgroups with candidate sectors:
  idle_end   last workgroup without candidates   end     cand / sig / sectors done, end (max)
  ref_*      k_refresh first start, last end     nhit, ncand  workgroups with candidates, sectors
  z_*        zone workgroup (thread 0): selection done, zone loaded, site deltas done, scan, survivors
             staged, window staged, zone stored (then flush)
  hit_p1/ver paired launches: the body's first merge's sectors done / the zone's verdict seen
             (zone_two's z_* stamps: loaded, merge-1 deltas, merge 1 in LDS, verdict, merge 2 in LDS, stored)
  period     k_body start to k_body start, per launch, inside a 128-merge step

usage: python tools/ktrace_show.py <dump file>
"""
import os
import sys

import numpy as np

EVERY, WG, SLOTS, HZ = 16, 2048, 12, 100e6


def main():
    raw = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 2 * WG, SLOTS)
    rows, t0abs, zrows = [], [], []
    for i in range(raw.shape[0]):
        body, ref, zw = raw[i, :WG - 8], raw[i, WG:], raw[i, WG - 8:WG]
        on = body[:, 0] > 0
        if not on.any():
            continue
        b = body[on].astype(np.float64)
        t0 = b[:, 0].min()
        us = lambda x: (x - t0) / HZ * 1e6
        role = body[on, 6] & 0xFF
        hit, idle, zone = role == 1, (role == 0) & (b[:, 5] > 0), role == 2
        r = ref[ref[:, 0] > 0].astype(np.float64)
        mx = lambda m, c: us(b[m, c].max()) if m.any() else np.nan
        t0abs.append((i * EVERY, t0))
        zwv = [[us(zw[w, k]) if zw[w, k] > 0 else np.nan for k in range(10)] for w in range(4)]
        zrows.append([i * EVERY] + [v for w in zwv for v in w])
        rows.append([i * EVERY, us(b[:, 0].max()), mx(b[:, 1] > 0, 1), mx(zone, 5), mx(idle, 5),
                     mx(hit, 2), mx(hit, 3), mx(hit, 4), mx(hit, 5),
                     us(r[:, 0].min()) if len(r) else np.nan, us(r[:, 5].max()) if len(r) else np.nan,
                     hit.sum(), (body[on, 6][hit] >> 8).sum(), on.sum(),
                     mx(zone, 1), mx(zone, 2), mx(zone, 3), mx(zone, 7), mx(zone, 8), mx(zone, 9), mx(zone, 4),
                     mx(hit & (b[:, 10] > 0), 10), mx(hit & (b[:, 11] > 0), 11), mx(zone, 10), mx(zone, 11)])
    # the merge period inside a step: first k_body start to the one EVERY merges later
    per = {m: np.nan for m, _ in t0abs}
    for (m0, t0), (m1, t1) in zip(t0abs[:-1], t0abs[1:]):
        if m1 - m0 == EVERY and m0 // 128 == m1 // 128:
            per[m0] = (t1 - t0) / HZ * 1e6 / EVERY
    for r in rows:
        r.append(per.get(r[0], np.nan))
    a = np.array(rows)
    names = ["start_max", "sel", "zone", "idle_end", "hit_cand", "hit_sig", "hit_sect", "hit_end", "ref_start",
             "ref_end", "nhit", "ncand", "nwg", "z_sel", "z_load", "z_sites", "z_scan", "z_keep", "z_win", "z_wrote",
             "hit_p1", "hit_ver", "z_masks", "z_tail", "period"]
    edges = [int(e) for e in os.environ.get("EDGES", "0,150,300,500,1000,2000,4000,8000,16000,24000,40000").split(",")]
    print(f"{'merges':<13}{'n':>5}" + "".join(f"{k:>10}" for k in names))
    for lo, hi in zip(edges[:-1], edges[1:]):
        sel = (a[:, 0] >= lo) & (a[:, 0] < hi)
        if not sel.any():
            continue
        med = [np.nanmedian(a[sel, j]) if np.isfinite(a[sel, j]).any() else np.nan for j in range(1, a.shape[1])]
        print(f"{lo:>6}-{hi:<6}{int(sel.sum()):>5}" + "".join(f"{v:>10.2f}" for v in med))
    if zrows:
        zone_waves(zrows, edges)



def zone_waves(zrows, edges):
    """zone_two's per-wave stamps (KTW: 0 loaded, 1 masks, 2 tail, 3 rel, 4 wb2, 5 scan written,
    6 after the scan barrier, 7 assembled, 8 window start, 9 window done), medians per bucket"""
    a = np.array(zrows)
    for lo, hi in zip(edges[:-1], edges[1:]):
        sel = (a[:, 0] >= lo) & (a[:, 0] < hi)
        if not sel.any() or np.isnan(a[sel, 1:]).all():
            continue
        med = np.nanmedian(a[sel, 1:], axis=0).reshape(4, 10)
        print(f"zone waves {lo}-{hi}:")
        for w in range(4):
            print("   wave %d " % w + " ".join("%6.2f" % v for v in med[w]))

if __name__ == "__main__":
    main()

