# A/B: the k_refresh grid of late steps (zone fits the 256-thread k_body): unchanged (2 per CU)
# vs GBPE_REFRESH_LATE=64 / 128 workgroups; every run's merges compared with its fixture
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
L=gpu-bpe_amd/lib/libgpubpe.so
AB_ROUNDS=2 timeout -k 10 850 python tools/ab_libs.py $L $L:GBPE_REFRESH_LATE=64 $L:GBPE_REFRESH_LATE=128 -- en1g c2 code1g > gpurun_out/r3c/ab_refresh_late.txt 2>&1
cat gpurun_out/r3c/ab_refresh_late.txt
