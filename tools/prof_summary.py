"""Summarise a rocprofv3 --kernel-trace run (rocpd SQLite .db or CSV dir).

usage: python tools/prof_summary.py <outdir> [--by-index KERNEL BUCKET]
Prints per-kernel launches / avg / total like rocprofv3 --stats; with
--by-index, the avg duration of KERNEL per BUCKET consecutive launches.
"""
import csv
import glob
import os
import sqlite3
import sys


def load(outdir):
    """Return [(kernel_name, start_ns, end_ns)] in dispatch order."""
    dbs = glob.glob(os.path.join(outdir, "*.db"))
    if dbs:
        c = sqlite3.connect(dbs[0])
        names = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
        kd = next(t for t in names if t.startswith("rocpd_kernel_dispatch"))
        ks = next(t for t in names if t.startswith("rocpd_info_kernel_symbol"))
        return c.execute(f"select s.kernel_name, d.start, d.end from {kd} d join {ks} s "
                         f"on d.kernel_id = s.id order by d.start").fetchall()
    rows = []
    for f in glob.glob(os.path.join(outdir, "*kernel_trace.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort(key=lambda r: r[1])
    return rows


def short(name):
    for tok in ("k_delta", "k_compact", "k_refresh", "k_select", "k_count_full", "k_symbols",
                "k_clear_dirty_all", "k_trie_walk", "k_chunk_scan1", "k_chunk_scan2",
                "k_chunk_compact", "k_dump_pairs", "k_export_symbols"):
        if tok in name:
            return tok
    return name[:40]


def main():
    rows = load(sys.argv[1])
    agg = {}
    for n, s, e in rows:
        a = agg.setdefault(short(n), [0, 0])
        a[0] += 1
        a[1] += e - s
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':<22}{'calls':>8}{'avg_us':>10}{'total_ms':>11}{'pct':>7}")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:<22}{c:>8}{t / c / 1e3:>10.2f}{t / 1e6:>11.2f}{100 * t / tot:>7.1f}")
    if "--by-index" in sys.argv:
        i = sys.argv.index("--by-index")
        kern, bucket = sys.argv[i + 1], int(sys.argv[i + 2])
        d = [e - s for n, s, e in rows if short(n) == kern]
        for b in range(0, len(d), bucket):
            seg = d[b:b + bucket]
            print(f"{kern}[{b}:{b + len(seg)}] avg {sum(seg) / len(seg) / 1e3:.2f} us")


if __name__ == "__main__":
    main()
