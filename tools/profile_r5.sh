# Round-5 profiles (one GPU call), every step with its own time limit:
#   1. kernel durations of one en1g run under rocprofv3 --kernel-trace --stats
#   2. (unless STATS_ONLY) two --pmc passes (FETCH_SIZE, WRITE_SIZE) over one en1g run: k_body traffic
# OUT names the directory under gpurun_out/ (default r5prof).
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r5prof}
mkdir -p $O
cd /tmp
EXPLORE_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ks -o run -- python3 $R/tools/explore_1g.py ${WL:-en1g} > $O/ks.log 2>&1
cp $(find /tmp/ks -name "*kernel_stats.csv") $O/${WL:-en1g}_kernel_stats.csv
[ -n "$STATS_ONLY" ] && exit 0
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o run -- python3 $R/tools/explore_1g.py en1g > $O/pf.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o run -- python3 $R/tools/explore_1g.py en1g > $O/pw.log 2>&1
python3 $R/tools/pmc_r2.py kbody /tmp/pf /tmp/pw $O/pf.log $O/pmc_kbody.json
