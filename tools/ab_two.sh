# A/B of two library builds, alternating runs on one box: tools/ab_two.sh <libA> <libB> (paths under gpu-bpe_amd/lib)
for i in 1 2; do
  for v in "$1" "$2"; do
    GBPE_LIB=$PWD/gpu-bpe_amd/lib/$v/libgpubpe.so EXPLORE_REPS=1 timeout -k 10 200 python tools/explore_1g.py en1g c2 > gpurun_out/ab_${v//\//_}_$i.log 2>&1 || exit 1
  done
done
