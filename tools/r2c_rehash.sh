# in-loop table rehash: parity (growth tests, full C5 / C4-shard / C2 fixtures) and C5 timing A/B
set -e
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_full.py tests/test_gpu_parity.py -m gpu -x -q -k "grow or code1g or ml1g64k or c2_bench or sparse or table" --timeout 200 --timeout-method thread > gpurun_out/rehash_tests.log 2>&1
for spec in "on:GBPE_REHASH=1" "off:GBPE_REHASH=0" "on2:GBPE_REHASH=1"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs EXPLORE_REPS=1 timeout -k 10 200 python tools/explore_1g.py code1g > gpurun_out/rh_$name.log 2>&1
done
