# Session-4 measurement (one GPU call): the encode walk's scratch store bursts
# (qv1: one 16-byte store per vector, the round-4 walk; qv4a: bursts of 4 per lane;
# qs2 / lib: wave-wide bursts, 2 / 4 vectors per lane queue),
# alternating processes, C3 1 GiB;
# the token stream's sha256 must agree across the builds.  Then the GPU suite.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s4
mkdir -p $O
L=$PWD/gpu-bpe_amd/lib
for r in 1 2; do
  for lib in $L/qv1/libgpubpe.so $L/qv4a/libgpubpe.so $L/qs2/libgpubpe.so $L/libgpubpe.so; do
    timeout -k 10 240 python -u tools/encode_once.py 10 $lib >> $O/encode_qs_ab.txt 2>> $O/encode_qs_ab.err || { echo ENCFAIL; tail -20 $O/encode_qs_ab.err; exit 1; }
  done
done
cat $O/encode_qs_ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "encode or tokenize or trie or smoke" > $O/gpu_tests_encode.txt 2>&1 || { echo TESTFAIL; tail -30 $O/gpu_tests_encode.txt; exit 1; }
tail -3 $O/gpu_tests_encode.txt
