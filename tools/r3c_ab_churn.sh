# A/B: k_churn with 8 positions loaded per thread before their LDS adds (lib/ch8) vs HEAD (lib/head);
# every run's merges compared with its fixture
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
AB_ROUNDS=2 timeout -k 10 850 python tools/ab_libs.py gpu-bpe_amd/lib/head/libgpubpe.so gpu-bpe_amd/lib/ch8/libgpubpe.so -- en1g c2 code1g > gpurun_out/r3c/ab_churn.txt 2>&1
cat gpurun_out/r3c/ab_churn.txt
