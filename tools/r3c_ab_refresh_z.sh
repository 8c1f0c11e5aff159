# A/B: the zone length below which steps run k_refresh on 64 workgroups: the 256-thread k_body's
# zone (8K u16, default) vs 16K (every one-workgroup zone) vs 1M (the zone-segment steps too)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
L=gpu-bpe_amd/lib/libgpubpe.so
AB_ROUNDS=2 timeout -k 10 850 python tools/ab_libs.py $L $L:GBPE_REFRESH_LATE_Z=16384 $L:GBPE_REFRESH_LATE_Z=1048576 -- en1g c2 > gpurun_out/r3c/ab_refresh_z.txt 2>&1
cat gpurun_out/r3c/ab_refresh_z.txt
