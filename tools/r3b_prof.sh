# Kernel durations (rocprofv3 --kernel-trace --stats) of one full en1g and one code1g run with the
# in-tree library, defaults vs the byte-pair first count and the sampled word table switched off;
# then the new lexicon-size GPU test.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3b_prof
cd /tmp
for cfg in en1g code1g; do
  EXPLORE_REPS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_new_$cfg -o run -- python3 $R/tools/explore_1g.py $cfg > /tmp/p_new_$cfg.log 2>&1
  cp $(find /tmp/p_new_$cfg -name "*kernel_stats.csv") $R/gpurun_out/r3b_prof/${cfg}_new.csv
  GBPE_LEX_SIZE=0 GBPE_COUNT_BYTES=0 EXPLORE_REPS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_old_$cfg -o run -- python3 $R/tools/explore_1g.py $cfg > /tmp/p_old_$cfg.log 2>&1
  cp $(find /tmp/p_old_$cfg -name "*kernel_stats.csv") $R/gpurun_out/r3b_prof/${cfg}_old.csv
done
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_lexicon.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r3b_lexicon_test.txt 2>&1
tail -3 gpurun_out/r3b_lexicon_test.txt
