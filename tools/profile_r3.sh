# Round-3 counters (one GPU call):
#   1. FETCH_SIZE / WRITE_SIZE calibration on k_body's and the walk's access patterns
#      (tools/micro/fetch_cal.hip)                                  -> gpurun_out/r3_fetch_calibration.json
#   2. two --pmc passes over one full en1g run (k_body)             -> gpurun_out/r3_pmc_kbody.json
#   3. two --pmc passes over one C3 encode                          -> gpurun_out/r3_pmc_encode.json
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/cf -o run -- $R/tools/micro/fetch_cal > /tmp/cf.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/cw -o run -- $R/tools/micro/fetch_cal > /tmp/cw.log 2>&1
python3 $R/tools/fetch_cal.py /tmp/cf /tmp/cw /tmp/cf.log $R/gpurun_out/r3_fetch_calibration.json
[ -n "$CAL_ONLY" ] && exit 0
if [ -z "$STATS_ONLY" ]; then
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o run -- python3 $R/tools/explore_1g.py en1g > /tmp/pf.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o run -- python3 $R/tools/explore_1g.py en1g > /tmp/pw.log 2>&1
python3 $R/tools/pmc_r2.py kbody /tmp/pf /tmp/pw /tmp/pf.log $R/gpurun_out/r3_pmc_kbody.json
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/ef -o run -- python3 $R/tools/encode_once.py 2 > /tmp/ef.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/ew -o run -- python3 $R/tools/encode_once.py 2 > /tmp/ew.log 2>&1
python3 $R/tools/pmc_r2.py encode /tmp/ef /tmp/ew /tmp/ef.log $R/gpurun_out/r3_pmc_encode.json
fi
# 4. kernel durations of one en1g run under rocprofv3 (bench.py puts k_body's beside its HIP-event figure)
EXPLORE_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ks -o run -- python3 $R/tools/explore_1g.py en1g > /tmp/ks.log 2>&1
cp $(find /tmp/ks -name "*kernel_stats.csv") $R/gpurun_out/r3_rocprof_en1g_kernel_stats.csv
