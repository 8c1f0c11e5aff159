# rocprofv3 kernel-trace stats of the bench (csv; the per-dispatch trace stays on the box)
set -e
export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/final_prof -o run -- python3 bench.py --no-cpu --steps 2 > gpurun_out/final_bench_rocprof.json 2> gpurun_out/final_bench_rocprof.err
mkdir -p gpurun_out/final_prof
find /tmp/final_prof -name '*stats.csv' -exec cp {} gpurun_out/final_prof/ \;
ls -la gpurun_out/final_prof
