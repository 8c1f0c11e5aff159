# kernel-trace A/B of two library builds on one box: tools/ab_prof.sh <libA> <libB> [config]
C=${3:-en1g}
for v in "$1" "$2"; do
  GBPE_LIB=$PWD/gpu-bpe_amd/lib/$v/libgpubpe.so SKIP_PMC=1 bash tools/profile_1g.sh $C || exit 1
  cp gpurun_out/mp_$C.txt gpurun_out/abp_${v}_$C.txt
done
