# sparse-entry threshold sweep of the C2 training leg (one GPU call); then a
# per-merge kernel profile of one setting
set -e
export TMPDIR=/tmp
for d in ${DIVS:-4294967295 64 256 1024 4096}; do
  GBPE_SPARSE_DIV=$d timeout -k 10 200 python bench.py --no-encode --no-cpu > gpurun_out/sweep_$d.json 2> gpurun_out/sweep_$d.err
  echo "div=$d done"
done
if [ -n "$PROF_DIV" ]; then
  R=$GRAFT_REPO_ROOT
  cd /tmp && GBPE_SPARSE_DIV=$PROF_DIV BENCH_DUMP_MERGES=/tmp/m.npy timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof -o run -- python3 $R/bench.py --no-encode --no-cpu > /tmp/b.log 2>&1
  cd $R && python tools/merge_profile.py /tmp/prof /tmp/m.npy > gpurun_out/mp_$PROF_DIV.txt 2>&1
fi
