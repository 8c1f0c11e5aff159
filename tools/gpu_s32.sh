# Session-32 A/B (one GPU call): k_churn's workgroup cap for the large early zones
# (GBPE_DEBUG chmax = 256, round 4, vs 512, the new default), fixtures checked.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s32
mkdir -p $O
L=gpu-bpe_amd/lib/libgpubpe.so
AB_REPS=2 AB_ROUNDS=2 timeout -k 10 700 python -u tools/ab_libs.py "$L:GBPE_DEBUG=chmax=256" "$L" -- en1g code1g ml1g64k > $O/ab.txt 2>&1 || { echo ABFAIL; tail -30 $O/ab.txt; exit 1; }
grep -E "^(en1g|code1g|ml1g64k) " $O/ab.txt
