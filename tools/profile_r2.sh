# Round-2 measurement of the bench workload (one GPU call), in this order:
#   1. two --pmc passes (FETCH_SIZE, WRITE_SIZE) over one full en1g run -> gpurun_out/r2_pmc_kbody.json
#   2. two --pmc passes over one C3 encode                                -> gpurun_out/r2_pmc_encode.json
#      (both copied into profiles/ on the box, where bench.py reads them)
#   3. bench.py default line                                              -> gpurun_out/r2_bench.json
#   4. rocprofv3 --kernel-trace --stats of the same command               -> gpurun_out/r2_prof/
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r2_prof
cd /tmp
if [ -z "$SKIP_PMC" ]; then
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o run -- python3 $R/tools/explore_1g.py en1g > /tmp/pf.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o run -- python3 $R/tools/explore_1g.py en1g > /tmp/pw.log 2>&1
python3 $R/tools/pmc_r2.py kbody /tmp/pf /tmp/pw /tmp/pf.log $R/gpurun_out/r2_pmc_kbody.json
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/ef -o run -- python3 $R/tools/encode_once.py 2 > /tmp/ef.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/ew -o run -- python3 $R/tools/encode_once.py 2 > /tmp/ew.log 2>&1
python3 $R/tools/pmc_r2.py encode /tmp/ef /tmp/ew /tmp/ef.log $R/gpurun_out/r2_pmc_encode.json
cp $R/gpurun_out/r2_pmc_kbody.json $R/gpurun_out/r2_pmc_encode.json $R/profiles/
fi
[ -n "$SKIP_BENCH" ] || timeout -k 10 500 python3 $R/bench.py > $R/gpurun_out/r2_bench.json 2> $R/gpurun_out/r2_bench.err
if [ -z "$SKIP_STATS" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pstats -o run -- python3 $R/bench.py > /tmp/pstats.log 2>&1
cp /tmp/pstats.log $R/gpurun_out/r2_bench_under_rocprof.json
cp $(find /tmp/pstats -name "*stats.csv") $R/gpurun_out/r2_prof/
fi
