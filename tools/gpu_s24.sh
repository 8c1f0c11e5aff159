# Session-24 A/B (one GPU call): the late k_refresh grid (GBPE_DEBUG rfl = 16, 32,
# 64 = default, 128; below 64 the WIDE form) on 1 GiB and C2, fixtures checked.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s24
mkdir -p $O
L=gpu-bpe_amd/lib/libgpubpe.so
AB_REPS=2 AB_ROUNDS=2 timeout -k 10 800 python -u tools/ab_libs.py "$L:GBPE_DEBUG=rfl=16" "$L:GBPE_DEBUG=rfl=32" "$L" "$L:GBPE_DEBUG=rfl=128" -- en1g c2 > $O/ab_rfl.txt 2>&1 || { echo ABFAIL; tail -30 $O/ab_rfl.txt; exit 1; }
grep -E "^(en1g|c2) " $O/ab_rfl.txt
