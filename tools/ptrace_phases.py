#!/usr/bin/env python3
"""Per-phase time of training runs from GBPE_DEBUG=ptrace=1 lines (tools/ab_libs.py
with AB_STDERR=1): merges, host wall ms and us/merge per k_body form."""
import re
import sys

for path in sys.argv[1:]:
    runs, cur, lib = [], [], None
    for line in open(path):
        if "[ptrace]" not in line:
            continue
        head, _, tail = line.partition("[ptrace]")
        d = {k: float(v) for k, v in re.findall(r"(\w+) ([\d.]+)", tail)}
        if cur and (d["merge"] < cur[-1]["merge"] or head != lib):
            runs.append((lib, cur))
            cur = []
        lib = head
        cur.append(d)
    if cur:
        runs.append((lib, cur))
    for lib, run in runs:
        print("%s total %.1f ms, %d merges" % (lib.strip(), sum(r["us"] for r in run) / 1e3, sum(r["done"] for r in run)))
        ph = {}
        for r in run:
            key = (min(int(r["zone1"]), 3), int(r["bt"]))
            p = ph.setdefault(key, [0.0, 0, 0, 1e18, 0])
            p[0] += r["us"]
            p[1] += r["done"]
            p[2] += r["paired"]
            p[3] = min(p[3], r["merge"])
            p[4] = max(p[4], r["merge"] + r["done"])
        for k, p in sorted(ph.items(), key=lambda kv: kv[1][3]):
            print("  zone1 %d bt %4d: merges %6d-%6d %7.1f ms %7.2f us/merge, paired %d" %
                  (k[0], k[1], p[3], p[4], p[0] / 1e3, p[0] / max(p[1], 1), p[2]))
