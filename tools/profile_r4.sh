# Round-4 profiles (one GPU call), every step with its own time limit:
#   1. kernel durations of one en1g run under rocprofv3 --kernel-trace --stats
#   2. two --pmc passes (FETCH_SIZE, WRITE_SIZE) over one en1g run: k_body traffic
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4prof
cd /tmp
EXPLORE_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ks -o run -- python3 $R/tools/explore_1g.py en1g > $R/gpurun_out/r4prof/ks.log 2>&1
cp $(find /tmp/ks -name "*kernel_stats.csv") $R/gpurun_out/r4prof/en1g_kernel_stats.csv
[ -n "$STATS_ONLY" ] && exit 0
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o run -- python3 $R/tools/explore_1g.py en1g > $R/gpurun_out/r4prof/pf.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o run -- python3 $R/tools/explore_1g.py en1g > $R/gpurun_out/r4prof/pw.log 2>&1
python3 $R/tools/pmc_r2.py kbody /tmp/pf /tmp/pw $R/gpurun_out/r4prof/pf.log $R/gpurun_out/r4prof/pmc_kbody.json
