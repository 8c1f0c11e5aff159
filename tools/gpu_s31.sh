# Session-31 profile (one GPU call): the C3 encode kernels under the kernel trace
# (durations) and two PMC passes (FETCH_SIZE, WRITE_SIZE) for their HBM traffic.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s31
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/enc -o run -- python3 $R/tools/encode_once.py 10 > $O/enc.log 2>&1 || { echo ENCFAIL; tail -20 $O/enc.log; exit 1; }
cp $(find /tmp/enc -name "*kernel_stats.csv") $O/c3_encode_kernel_stats.csv
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/encf -o run -- python3 $R/tools/encode_once.py 3 > $O/encf.log 2>&1 || { echo PMCF; tail -20 $O/encf.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/encw -o run -- python3 $R/tools/encode_once.py 3 > $O/encw.log 2>&1 || { echo PMCW; tail -20 $O/encw.log; exit 1; }
for k in k_trie_walk_v5 k_chunk_compact4; do
  for d in encf encw; do echo "== $d $k" >> $O/c3_encode_pmc.txt; python3 $R/tools/pmc_kernel_sum.py /tmp/$d $k >> $O/c3_encode_pmc.txt; done
done
cat $O/c3_encode_pmc.txt
grep -E "walk|compact4|scan" $O/c3_encode_kernel_stats.csv | cut -c1-200
