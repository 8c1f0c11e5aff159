# A/B of the k_refresh grid (GBPE_REFRESH_BLOCKS) on the 1 GiB headline and C2
export TMPDIR=/tmp
for spec in "r512:GBPE_REFRESH_BLOCKS=512" "r64:GBPE_REFRESH_BLOCKS=64" "r128:GBPE_REFRESH_BLOCKS=128" "r256:GBPE_REFRESH_BLOCKS=256" "r1024:GBPE_REFRESH_BLOCKS=1024" "r512b:GBPE_REFRESH_BLOCKS=512"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs EXPLORE_REPS=1 timeout -k 10 200 python tools/explore_1g.py en1g c2 > gpurun_out/rf_$name.log 2>&1 || exit 1
done
