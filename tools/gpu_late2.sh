# late loop: phase stamps of the en1g run (KTRACE build) after the parity checks of gpu_late1.sh
export TMPDIR=/tmp
GBPE_LIB=$PWD/gpu-bpe_amd/lib/kt/libgpubpe.so GBPE_KTRACE_OUT=/tmp/ktl AB_REPS=1 AB_ROUNDS=1 timeout -k 10 200 python -u tools/ab_libs.py gpu-bpe_amd/lib/kt/libgpubpe.so -- en1g > gpurun_out/r4_kt_late.txt 2>&1
f=$(ls -S /tmp/ktl.* | head -1)
python tools/ktrace_late.py $f > gpurun_out/r4_ktrace_late.txt
