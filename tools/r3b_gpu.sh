# Round-3 session B check on MI355X: the GPU suite with the in-tree library, then an A/B of the
# round's last build (lib/base) against the working tree (lib/cur) on the 1 GiB, C2 and code configurations.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3b_gpu_tests.txt 2>&1
tail -3 gpurun_out/r3b_gpu_tests.txt
AB_ROUNDS=1 timeout -k 10 500 python tools/ab_libs.py gpu-bpe_amd/lib/base/libgpubpe.so gpu-bpe_amd/lib/cur/libgpubpe.so -- en1g c2 code1g > gpurun_out/r3b_ab.txt 2>&1
cat gpurun_out/r3b_ab.txt
