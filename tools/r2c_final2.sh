set -e
bash tools/r2c_final.sh
export TMPDIR=/tmp
GBPE_LIB=$PWD/gpu-bpe_amd/lib/ldsrd/libgpubpe.so timeout -k 10 400 python -u -m pytest tests/test_gpu_full.py -m gpu -x -q -k "c2 or en1g or ml1g64k" --timeout 200 --timeout-method thread > gpurun_out/ldsrd_tests.log 2>&1
bash tools/ab_two.sh base ldsrd
