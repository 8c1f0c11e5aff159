# A/B: k_refresh with block 0's state snapshot in the flag load's round trip (lib/ref2), plus the
# merge committed by an extra k_body workgroup (lib/ref3), vs HEAD (lib/head)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ROUNDS=2 timeout -k 10 850 python tools/ab_libs.py gpu-bpe_amd/lib/head/libgpubpe.so gpu-bpe_amd/lib/ref2/libgpubpe.so gpu-bpe_amd/lib/ref3/libgpubpe.so -- en1g c2 code1g > gpurun_out/r3b_ab_refresh.txt 2>&1
cat gpurun_out/r3b_ab_refresh.txt
