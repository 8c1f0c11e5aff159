"""HBM traffic per k_body launch from two rocprofv3 --pmc passes of
`bench.py --no-encode --no-cpu --no-kernel-timing` (FETCH_SIZE and WRITE_SIZE
collected separately, MI355X_MICROARCH.md §HBM), next to the bytes k_body
itself counts (train_detail.body_bytes_run of the same command's JSON line).

FETCH_SIZE/WRITE_SIZE are KiB.  Reads are doubled (the guide's gfx950 rule for
wide streaming reads); k_body's reads are mostly narrow gathers, so the raw
(undoubled) figure is reported too.

usage: python tools/pmc_kbody.py <fetch dir> <write dir> <bench json> [out.json]
"""
import csv
import glob
import json
import os
import sys


def series(d, counter):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
        vals += [float(r["Counter_Value"]) * 1024.0 for r in rows
                 if r["Counter_Name"] == counter and "k_body" in r["Kernel_Name"]]
    return vals


def main():
    fd, wd, bj = sys.argv[1:4]
    line = json.loads(open(bj).read().strip().splitlines()[-1])
    td = line["train_detail"]
    n = int(td["sparse"]["merges"])
    fetch, write = series(fd, "FETCH_SIZE")[-n:], series(wd, "WRITE_SIZE")[-n:]
    k = min(len(fetch), len(write))
    raw = sum(fetch[-k:]) / k
    wr = sum(write[-k:]) / k
    alg = td["body_bytes_run"] / n
    out = {"launches": k, "fetch_bytes_raw_per_launch": raw, "read_bytes_per_launch": 2 * raw,
           "write_bytes_per_launch": wr, "hbm_bytes_per_launch": 2 * raw + wr,
           "hbm_bytes_raw_per_launch": raw + wr, "algorithmic_bytes_per_launch": alg,
           "traffic_over_algorithmic": (2 * raw + wr) / alg}
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 4:
        open(sys.argv[4], "w").write(s + "\n")


if __name__ == "__main__":
    main()
