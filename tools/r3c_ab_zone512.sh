# A/B: zones of 8K-16K symbols in a 512-thread k_body (32 zone symbols per thread, GBPE_ZONE512=1)
# vs the 1024-thread forms; every run's merges compared with its fixture
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
L=gpu-bpe_amd/lib/z512/libgpubpe.so
AB_ROUNDS=2 timeout -k 10 850 python tools/ab_libs.py $L $L:GBPE_ZONE512=1 -- en1g c2 code1g > gpurun_out/r3c/ab_zone512.txt 2>&1
cat gpurun_out/r3c/ab_zone512.txt
