# Session-21 A/B (one GPU call): k_body workgroups per bitmap word for rows of few
# words (GBPE_DEBUG bsub = 1, 2, 4), merges checked against the fixtures.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s21
mkdir -p $O
L=gpu-bpe_amd/lib/libgpubpe.so
AB_REPS=3 AB_ROUNDS=2 timeout -k 10 900 python -u tools/ab_libs.py "$L:GBPE_DEBUG=bsub=1" "$L:GBPE_DEBUG=bsub=2" "$L:GBPE_DEBUG=bsub=4" -- c1 c2 en1g > $O/ab.txt 2>&1 || { echo ABFAIL; tail -30 $O/ab.txt; exit 1; }
grep -E "^(c1|c2|en1g) " $O/ab.txt
