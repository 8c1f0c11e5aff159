# Round-3 session B, second check: the GPU suite with the in-tree library (byte-pair first
# count, sampled word-table size), then an A/B against the previous commit's build (lib/cur),
# the new build with either change switched off, and 8-merge sub-steps.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3b2_gpu_tests.txt 2>&1
tail -3 gpurun_out/r3b2_gpu_tests.txt
AB_ROUNDS=1 timeout -k 10 500 python tools/ab_libs.py gpu-bpe_amd/lib/cur/libgpubpe.so gpu-bpe_amd/lib/cur2/libgpubpe.so \
  gpu-bpe_amd/lib/cur2/libgpubpe.so:GBPE_LEX_SIZE=0 gpu-bpe_amd/lib/cur2/libgpubpe.so:GBPE_COUNT_BYTES=0 \
  gpu-bpe_amd/lib/cur2/libgpubpe.so:GBPE_SUBSTEP=8 -- en1g code1g > gpurun_out/r3b2_ab.txt 2>&1
cat gpurun_out/r3b2_ab.txt
