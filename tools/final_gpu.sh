set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt_all.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 timeout -k 10 300 python bench.py --sharded > gpurun_out/bench_sharded1.json 2> gpurun_out/bench_sharded1.err
GBPE_SPARSE_DIV=4294967295 timeout -k 10 300 python bench.py --no-encode --no-cpu > gpurun_out/bench_dense.json 2> gpurun_out/bench_dense.err
