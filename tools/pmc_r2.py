"""HBM traffic of one workload window from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, each its own run; MI355X_MICROARCH.md §HBM:
FETCH_SIZE doubled on gfx950 for wide streaming reads, WRITE_SIZE as is;
both are KiB).  The raw (undoubled) read figure is kept beside it: k_body's
reads are mostly narrow gathers, for which the doubling is uncalibrated.

  kbody:  python tools/pmc_r2.py kbody <fetch dir> <write dir> <explore json line file> <out.json>
          window = one full en1g training run (tools/explore_1g.py en1g); algorithmic bytes
          per launch = that run's k_body byte counter / its k_body launches (sparse merges
          minus paired merges)
  encode: python tools/pmc_r2.py encode <fetch dir> <write dir> <encode json file> <out.json>
          window = one C3 encode (tools/encode_once.py); algorithmic bytes n + 4T
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, names):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and any(k in r["Kernel_Name"] for k in names):
                vals[int(r["Dispatch_Id"])] = vals.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"]) * 1024.0
    return [vals[k] for k in sorted(vals)]


def main():
    mode, fd, wd, jf, out = sys.argv[1:6]
    info = json.loads([ln for ln in open(jf).read().splitlines() if ln.startswith("{")][-1])
    if mode == "kbody":
        # k_body launches of the run: one per sparse merge, one per pair of a paired launch
        n = int(info["stats"]["sparse_merges"]) - int(info["stats"].get("paired_merges", 0))
        fetch, write = per_dispatch(fd, "FETCH_SIZE", ["k_body"])[-n:], per_dispatch(wd, "WRITE_SIZE", ["k_body"])[-n:]
        k = min(len(fetch), len(write))
        raw, wr = sum(fetch[-k:]) / k, sum(write[-k:]) / k
        alg = info["stats"]["body_bytes"] / n
        res = {"workload": "en1g-full-run", "kernel": "k_body", "launches": k,
               "fetch_bytes_raw_per_launch": raw, "read_bytes_per_launch": 2 * raw, "write_bytes_per_launch": wr,
               "hbm_bytes_per_launch": 2 * raw + wr, "hbm_bytes_raw_per_launch": raw + wr,
               "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": (2 * raw + wr) / alg,
               "raw_over_algorithmic": (raw + wr) / alg}
    else:
        names = ["k_trie_walk", "k_chunk_scan", "k_chunk_compact", "k_enc"]
        fetch, write = per_dispatch(fd, "FETCH_SIZE", names), per_dispatch(wd, "WRITE_SIZE", names)
        reps = int(info["reps"])
        raw, wr = sum(fetch) / reps, sum(write) / reps
        alg = info["bytes"] + 4 * info["tokens"]
        res = {"workload": "c3-1g", "chunk_size": info["chunk_size"], "kernels": names, "encodes": reps,
               "fetch_bytes_raw_per_encode": raw, "read_bytes_per_encode": 2 * raw, "write_bytes_per_encode": wr,
               "hbm_bytes_per_encode": 2 * raw + wr, "algorithmic_bytes": alg,
               "traffic_over_algorithmic": (2 * raw + wr) / alg}
    s = json.dumps(res, indent=1)
    print(s)
    open(out, "w").write(s + "\n")


if __name__ == "__main__":
    main()
