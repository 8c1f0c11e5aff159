# Instruction-cache behaviour of the late sparse loop (diagnostic): two
# rocprofv3 --pmc passes over one full en1g run; per-dispatch averages of
# k_body and k_refresh over the last 10,000 launches of each.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
i=0
for set in "SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d /tmp/pi$i -o run -- python3 $R/tools/explore_1g.py en1g > /tmp/pi$i.log 2>&1 || { echo "pass $i failed"; tail -5 /tmp/pi$i.log; }
done
python3 - <<'PY' > $R/gpurun_out/pmc_icache.txt
import csv, glob
for i in (1, 2):
    per = {}
    for f in glob.glob(f"/tmp/pi{i}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"]
            k = "k_body" if "k_body" in kn else "k_refresh" if "k_refresh" in kn else None
            if k:
                d = per.setdefault((k, r["Counter_Name"]), {})
                d[int(r["Dispatch_Id"])] = d.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    for (k, c), d in sorted(per.items()):
        v = [d[x] for x in sorted(d)][-10000:]
        print(k, c, "launches", len(d), "avg_last10k", round(sum(v) / max(1, len(v)), 1))
PY
cat $R/gpurun_out/pmc_icache.txt
