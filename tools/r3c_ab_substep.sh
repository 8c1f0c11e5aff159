# A/B: sub-step length while the zone exceeds 1M symbols (16, default) vs 8 and 32, and the
# sub-step zone threshold at 4M; every run's merges compared with its fixture
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
L=gpu-bpe_amd/lib/libgpubpe.so
AB_ROUNDS=2 timeout -k 10 850 python tools/ab_libs.py $L $L:GBPE_SUBSTEP=8 $L:GBPE_SUBSTEP=32 $L:GBPE_SUBSTEP_ZONE=4194304 -- en1g c2 > gpurun_out/r3c/ab_substep.txt 2>&1
cat gpurun_out/r3c/ab_substep.txt
