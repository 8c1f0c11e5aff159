# Round profile of the bench workload (one GPU call):
#   1. the default bench line (the judged command)            -> gpurun_out/bench.json
#   2. rocprofv3 --kernel-trace --stats of the same command    -> gpurun_out/prof_stats/
#   3. two --pmc passes (FETCH_SIZE, WRITE_SIZE) of the train leg -> profiles/r1_pmc_kbody.json
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
[ -n "$SKIP_BENCH" ] || timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pstats -o run -- python3 $R/bench.py > /tmp/pstats.log 2>&1
cp /tmp/pstats.log $R/gpurun_out/bench_under_rocprof.json
mkdir -p $R/gpurun_out/prof_stats && cp $(find /tmp/pstats -name "*stats.csv") $R/gpurun_out/prof_stats/
timeout -k 10 300 python3 $R/bench.py --no-encode --no-cpu --no-kernel-timing > /tmp/pmcref.json 2>/dev/null
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o run -- python3 $R/bench.py --no-encode --no-cpu --no-kernel-timing > /tmp/pf.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o run -- python3 $R/bench.py --no-encode --no-cpu --no-kernel-timing > /tmp/pw.log 2>&1
cd $R
grep "^{\"metric\"" /tmp/pf.log | tail -1 > gpurun_out/pmc_bench.json
python tools/pmc_kbody.py /tmp/pf /tmp/pw gpurun_out/pmc_bench.json gpurun_out/pmc_kbody.json
