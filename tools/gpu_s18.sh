# Session-18 diagnostic (one GPU call): what a C1 run (256 KiB ASCII @ 1K) spends
# its 25 ms on — steps, dense/sparse merges, host split, kernel stats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s18
mkdir -p $O
GBPE_DEBUG=htime=1 timeout -k 10 120 python3 tools/c1_probe.py > $O/c1.log 2>&1 || { echo C1FAIL; tail -20 $O/c1.log; exit 1; }
cat $O/c1.log | cut -c1-900
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/c1 -o run -- python3 tools/c1_probe.py > $O/c1_prof.log 2>&1 || { echo PROFFAIL; tail -20 $O/c1_prof.log; exit 1; }
python3 tools/prof_summary.py /tmp/c1 > $O/c1_kernels.txt 2>&1 || true
head -25 $O/c1_kernels.txt
