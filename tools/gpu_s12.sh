# Session-12 diagnostic (one GPU call): run-to-run variance of the 1 GiB headline
# run — in one context (pooled buffers reused) and in fresh contexts (new device
# allocations each run) — in two processes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s12
mkdir -p $O
for p in 1 2; do
  timeout -k 10 400 python -u tools/var_probe.py 4 >> $O/var.txt 2>> $O/var.err || { echo VARFAIL; tail -20 $O/var.err; exit 1; }
done
cat $O/var.txt
