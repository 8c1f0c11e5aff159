# Session-20 A/B (one GPU call): k_body's minimum workgroup count for small
# stores (GBPE_DEBUG bmin; 1 = the round-4 sizing), C1 / C2 / 1 GiB / C5, merges
# checked against the fixtures.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s20
mkdir -p $O
L=gpu-bpe_amd/lib/libgpubpe.so
AB_REPS=3 AB_ROUNDS=2 timeout -k 10 900 python -u tools/ab_libs.py "$L:GBPE_DEBUG=bmin=1" "$L:GBPE_DEBUG=bmin=16" "$L:GBPE_DEBUG=bmin=32" "$L:GBPE_DEBUG=bmin=64" -- c1 c2 en1g code1g > $O/ab.txt 2>&1 || { echo ABFAIL; tail -30 $O/ab.txt; exit 1; }
grep -E "^(c1|c2|en1g|code1g) " $O/ab.txt
