# A/B runs of the C2 training leg: each argument is "name:ENV=V,ENV2=V2"
set -e
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 200 python bench.py --no-encode --no-cpu > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
  echo "$name done"
done
