# Session-23 A/B (one GPU call): k_body's workgroup cap (GBPE_DEBUG bcap: 256 =
# one per CU, 512, 1024) on the large-row corpora, and the 1024-thread form for
# small zones too (z256=0) on 1 GiB / C2; merges checked against the fixtures.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s23
mkdir -p $O
L=gpu-bpe_amd/lib/libgpubpe.so
AB_REPS=2 AB_ROUNDS=2 timeout -k 10 500 python -u tools/ab_libs.py "$L:GBPE_DEBUG=bcap=256" "$L:GBPE_DEBUG=bcap=512" "$L:GBPE_DEBUG=bcap=1024" -- code1g ml1g64k > $O/ab_bcap.txt 2>&1 || { echo ABFAIL; tail -30 $O/ab_bcap.txt; exit 1; }
grep -E "^(code1g|ml1g64k) " $O/ab_bcap.txt
AB_REPS=2 AB_ROUNDS=2 timeout -k 10 500 python -u tools/ab_libs.py "$L" "$L:GBPE_DEBUG=z256=0" -- en1g c2 c1 > $O/ab_z256.txt 2>&1 || { echo ABFAIL2; tail -30 $O/ab_z256.txt; exit 1; }
grep -E "^(en1g|c2|c1) " $O/ab_z256.txt
