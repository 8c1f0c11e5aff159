# Round-3 closing run at HEAD: the GPU suite, smoke, the default bench line, rocprof kernel
# stats of the bench, and k_body's HBM traffic (FETCH_SIZE / WRITE_SIZE passes) for the bench's
# roofline.traffic.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c_gpu_tests.txt 2>&1
tail -2 gpurun_out/r3c_gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3c_smoke.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.err
tail -c 300 gpurun_out/r3c_bench.json
cd /tmp
EXPLORE_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/c_ks -o run -- python3 $R/tools/explore_1g.py en1g > /tmp/c_ks.log 2>&1
mkdir -p $R/gpurun_out/r3c_prof
cp $(find /tmp/c_ks -name "*kernel_stats.csv") $R/gpurun_out/r3c_prof/en1g_kernel_stats.csv
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/c_pf -o run -- python3 $R/tools/explore_1g.py en1g > /tmp/c_pf.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/c_pw -o run -- python3 $R/tools/explore_1g.py en1g > /tmp/c_pw.log 2>&1
python3 $R/tools/pmc_r2.py kbody /tmp/c_pf /tmp/c_pw /tmp/c_pf.log $R/gpurun_out/r3c_pmc_kbody.json
