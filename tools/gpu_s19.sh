# Session-19 diagnostic (one GPU call): C1's merge phases (ktrace build).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s19
mkdir -p $O
GBPE_LIB=$PWD/gpu-bpe_amd/lib/kt/libgpubpe.so GBPE_KTRACE_OUT=/tmp/kt_c1 timeout -k 10 120 python3 tools/c1_probe.py > $O/kt_c1.log 2>&1 || { echo KTFAIL; tail -20 $O/kt_c1.log; exit 1; }
f=$(ls -t /tmp/kt_c1.* | head -1)
EDGES=0,64,128,256,384,512,640,768 python3 tools/ktrace_show.py $f > $O/ktrace_c1.txt
cat $O/ktrace_c1.txt
