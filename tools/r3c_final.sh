# Round-3 closing run at HEAD: the GPU suite, smoke, k_body's rocprof kernel stats over one 1 GiB
# run (the bench line's rocprof_us_per_launch reads them), then the default bench line.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c profiles/r3c
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c/final_gpu_tests.txt 2>&1
tail -2 gpurun_out/r3c/final_gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3c/final_smoke.txt 2>&1
tail -1 gpurun_out/r3c/final_smoke.txt
cd /tmp
EXPLORE_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/f_ks -o run -- python3 $R/tools/explore_1g.py en1g > /tmp/f_ks.log 2>&1
cp $(find /tmp/f_ks -name "*kernel_stats.csv") $R/profiles/r3c/en1g_kernel_stats.csv
cp $R/profiles/r3c/en1g_kernel_stats.csv $R/gpurun_out/r3c/en1g_kernel_stats.csv
cd $R
timeout -k 10 600 python bench.py > gpurun_out/r3c/final_bench.json 2> gpurun_out/r3c/final_bench.err
tail -c 300 gpurun_out/r3c/final_bench.json
