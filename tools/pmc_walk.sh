# Cache / stall counters of the encode walk (diagnostic), one rocprofv3 --pmc pass each.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
i=0
for set in "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d /tmp/pw$i -o run -- python3 $R/tools/encode_once.py 1 > /tmp/pw$i.log 2>&1 || { echo "pass $i failed"; tail -5 /tmp/pw$i.log; }
done
python3 - <<'PY' > $R/gpurun_out/pmc_walk.txt
import csv, glob
for i in (1, 2, 3):
    tot = {}
    for f in glob.glob(f"/tmp/pw{i}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r["Kernel_Name"]
            k = "walk" if "walk" in kn else "compact" if "compact" in kn else None
            if k:
                key = (k, r["Counter_Name"])
                tot[key] = tot.get(key, 0.0) + float(r["Counter_Value"])
    for k, v in sorted(tot.items()):
        print(k[0], k[1], f"{v:.4g}")
PY
cat $R/gpurun_out/pmc_walk.txt
