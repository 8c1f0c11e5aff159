# A/B of the dense zone k_delta tiles-per-workgroup knob on the 1 GiB headline
export TMPDIR=/tmp
for spec in "tpw8:GBPE_DELTA_TPW=8" "tpw16:GBPE_DELTA_TPW=16" "tpw32:GBPE_DELTA_TPW=32" "mt0:GBPE_DELTA_MT=0" "tpw8b:GBPE_DELTA_TPW=8"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs EXPLORE_REPS=1 timeout -k 10 200 python tools/explore_1g.py en1g > gpurun_out/tpw_$name.log 2>&1 || exit 1
done
