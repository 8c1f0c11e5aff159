# Session-30 A/B (one GPU call): zone segments from 8K-symbol zones up (GBPE_DEBUG
# zslo=8192: zones of 8K-16K as two 8K segments instead of zone_one's 1024 x 16).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s30
mkdir -p $O
L=gpu-bpe_amd/lib/libgpubpe.so
AB_REPS=2 AB_ROUNDS=2 timeout -k 10 700 python -u tools/ab_libs.py "$L" "$L:GBPE_DEBUG=zslo=8192" -- en1g c2 c1 > $O/ab.txt 2>&1 || { echo ABFAIL; tail -30 $O/ab.txt; exit 1; }
grep -E "^(en1g|c2|c1) " $O/ab.txt
