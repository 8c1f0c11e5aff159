"""HBM traffic per merge of the two stream kernels from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE collected separately, the MI355X guide's recipe), next
to the algorithmic bytes s*(2*N_i + N_{i+1}) of the same merges.

FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes
of a wide streaming read, so reads are doubled (MI355X_MICROARCH.md §HBM).

usage: python tools/pmc_traffic.py <fetch dir> <write dir> <merges.npy> <n0> <s> [out.json]
  merges.npy: BENCH_DUMP_MERGES of the same workload; n0: initial symbol count;
  s: bytes per symbol.  Uses the last K launches of each kernel, K = merges timed.
"""
import csv
import glob
import json
import os
import sys

import numpy as np

KERNELS = ("k_delta", "k_compact", "k_refresh", "k_select")


def series(d, counter):
    out = {k: [] for k in KERNELS}
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
        for r in rows:
            if r["Counter_Name"] != counter:
                continue
            for k in KERNELS:
                if k in r["Kernel_Name"]:
                    out[k].append(float(r["Counter_Value"]) * 1024.0)
    return {k: np.array(v) for k, v in out.items()}


def main():
    fd, wd, mpath, n0, s = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
    fetch, write = series(fd, "FETCH_SIZE"), series(wd, "WRITE_SIZE")
    k = min(len(fetch["k_delta"]), len(write["k_delta"]))
    # the timed run is the tail of the trace; its merge count is the launches after the warmup run
    m = np.load(mpath)
    timed = int(os.environ.get("PMC_TIMED_MERGES", "0")) or k
    counts = m[:timed, 3].astype(np.int64)
    n = n0 - np.concatenate([[0], np.cumsum(counts)])
    alg = s * (2 * n[:-1] + n[1:])
    res = {"merges": timed, "bytes_per_symbol": s,
           "algorithmic_bytes_per_merge": float(alg.mean())}
    for kn in KERNELS:
        f = fetch[kn][-timed:]
        w = write[kn][-timed:]
        res[kn] = {"fetch_bytes_raw": float(f.mean()), "read_bytes": float(2 * f.mean()),
                   "write_bytes": float(w.mean()), "hbm_bytes": float(2 * f.mean() + w.mean())}
    pair = res["k_delta"]["hbm_bytes"] + res["k_compact"]["hbm_bytes"]
    res["stream_pair_hbm_bytes_per_merge"] = pair
    res["traffic_over_algorithmic"] = pair / res["algorithmic_bytes_per_merge"]
    txt = json.dumps(res, indent=1)
    print(txt)
    if len(sys.argv) > 6:
        open(sys.argv[6], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
