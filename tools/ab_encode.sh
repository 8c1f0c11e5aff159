# A/B runs of the full bench (train + encode): each argument is "name:ENV=V,ENV2=V2"
set -e
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python bench.py --no-cpu > gpurun_out/abe_$name.json 2> gpurun_out/abe_$name.err
  echo "$name done"
done
