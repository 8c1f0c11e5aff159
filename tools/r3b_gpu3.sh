# GPU suite with the in-tree library, then kernel durations of one en1g and one code1g run
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3b_prof3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3b3_gpu_tests.txt 2>&1
tail -3 gpurun_out/r3b3_gpu_tests.txt
cd /tmp
for cfg in en1g code1g; do
  EXPLORE_REPS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p3_$cfg -o run -- python3 $R/tools/explore_1g.py $cfg > $R/gpurun_out/r3b_prof3/$cfg.log 2>&1
  cp $(find /tmp/p3_$cfg -name "*kernel_stats.csv") $R/gpurun_out/r3b_prof3/${cfg}.csv
done
