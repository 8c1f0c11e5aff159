"""Join the rocprofv3 FETCH_SIZE / WRITE_SIZE passes over tools/micro/fetch_cal
with the byte counts it printed: counter bytes per requested byte and per
distinct 128-B line, for each access pattern.

  python tools/fetch_cal.py <fetch dir> <write dir> <fetch_cal stdout> <out.json>
"""
import csv
import glob
import json
import os
import sys


def counters(d, name):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                out.setdefault(k, []).append(float(r["Counter_Value"]) * 1024.0)
    return out


def main():
    fd, wd, log, outp = sys.argv[1:5]
    spec = [json.loads(ln) for ln in open(log) if ln.startswith("{")]
    fetch, write = counters(fd, "FETCH_SIZE"), counters(wd, "WRITE_SIZE")
    rows = []
    for s in spec:
        k = s["kernel"]
        f = fetch.get(k, [None])[-1]
        w = write.get(k, [None])[-1]
        row = dict(s)
        if k == "k_stream16":   # the first k_stream16 launch is the cache eviction pass
            f = fetch.get(k, [None])[-1]
        row["fetch_bytes"] = f
        row["write_bytes"] = w
        for nm, v in (("fetch", f), ("write", w)):
            if v is not None:
                row[f"{nm}_per_requested_byte"] = round(v / s["requested"], 4)
                row[f"{nm}_per_line"] = round(v / s["lines"], 2)
        rows.append(row)
    res = {"tool": "tools/micro/fetch_cal.hip", "line_bytes": 128,
           "meaning": "counter bytes / requested bytes and / distinct 128-B lines touched, per access pattern",
           "patterns": rows}
    s = json.dumps(res, indent=1)
    print(s)
    open(outp, "w").write(s + "\n")


if __name__ == "__main__":
    main()
