# body_sector's cycle split per step (the -DGBPE_BSPROF build, tools/build_variant.sh bsp -DGBPE_BSPROF):
# C5's first 40 steps and a whole 1 GiB run; lines "[bsprof] ..." on stderr
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r4h
GBPE_BSPROF=1 GBPE_LIB=$PWD/gpu-bpe_amd/lib/bsp/libgpubpe.so EXPLORE_REPS=1 EXPLORE_MAX_STEPS=40 timeout -k 10 300 python tools/explore_1g.py code1g > gpurun_out/r4h/bsp_code1g.txt 2>&1
GBPE_BSPROF=1 GBPE_LIB=$PWD/gpu-bpe_amd/lib/bsp/libgpubpe.so EXPLORE_REPS=1 timeout -k 10 300 python tools/explore_1g.py en1g > gpurun_out/r4h/bsp_en1g.txt 2>&1
