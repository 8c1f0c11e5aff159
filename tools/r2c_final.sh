# Round-2 closing run: GPU tests, smoke, default bench (all legs), rocprof stats of the bench
# (the per-dispatch kernel trace stays in /tmp on the box: only the summaries come back)
set -e
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final_gt.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/final_prof -o run -- python3 bench.py --no-cpu --steps 2 > gpurun_out/final_bench_rocprof.json 2> gpurun_out/final_bench_rocprof.err
mkdir -p gpurun_out/final_prof && find /tmp/final_prof -name '*stats.csv' -exec cp {} gpurun_out/final_prof/ \;
