# A/B: k_body's stale-window copy with 8 loads in flight per thread + k_zdr reading a dump's flag and bounds together and 4 entries at a time (lib/cp8) vs HEAD (lib/z512),
# and cp8 with 256-thread body workgroups while the dense kernels run the zone (GBPE_DENSE256=1)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
AB_ROUNDS=2 timeout -k 10 850 python tools/ab_libs.py gpu-bpe_amd/lib/z512/libgpubpe.so gpu-bpe_amd/lib/cp8/libgpubpe.so gpu-bpe_amd/lib/cp8/libgpubpe.so:GBPE_DENSE256=1 -- en1g c2 code1g > gpurun_out/r3c/ab_copy.txt 2>&1
cat gpurun_out/r3c/ab_copy.txt
