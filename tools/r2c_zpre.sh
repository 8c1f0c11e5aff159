export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_sparse.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/zpre_tests.log 2>&1 && bash tools/ab_two.sh base zpre
