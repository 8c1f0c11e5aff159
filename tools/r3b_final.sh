# Round-3 closing measurements at HEAD: smoke, the default bench line, and the rocprof
# kernel stats of the bench (summaries only come back).  The GPU suite ran on this build
# in tools/r3b_gpu3.sh.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3b_final_smoke.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/r3b_final_bench.json 2> gpurun_out/r3b_final_bench.err
tail -c 600 gpurun_out/r3b_final_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/final_prof -o run -- python3 bench.py --no-cpu --steps 2 > gpurun_out/r3b_final_bench_rocprof.json 2> gpurun_out/r3b_final_bench_rocprof.err
mkdir -p gpurun_out/r3b_final_prof && find /tmp/final_prof -name '*stats.csv' -exec cp {} gpurun_out/r3b_final_prof/ \;
