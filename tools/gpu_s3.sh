# Session-3 measurements (one GPU call): (1) the encode walk with and without its
# scratch stores (lib/nostore: -DGBPE_WALK_NOSTORE, tokens not written), alternating
# processes, C3 1 GiB; (2) phase stamps of the late merge chain at 1 GiB and on C5
# (lib/kt: -DGBPE_KTRACE).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s3
mkdir -p $O
L=$PWD/gpu-bpe_amd/lib
for r in 1 2; do
  for lib in $L/libgpubpe.so $L/nostore/libgpubpe.so; do
    timeout -k 10 240 python -u tools/encode_once.py 10 $lib >> $O/encode_nostore_ab.txt 2>> $O/encode_nostore_ab.err || { echo ENCFAIL; tail -20 $O/encode_nostore_ab.err; exit 1; }
  done
done
cat $O/encode_nostore_ab.txt
for wl in en1g code1g; do
  GBPE_LIB=$L/kt/libgpubpe.so GBPE_KTRACE_OUT=/tmp/kt_$wl timeout -k 10 300 python -u tools/explore_1g.py $wl > $O/kt_$wl.log 2>&1 || { echo KTFAIL; tail -20 $O/kt_$wl.log; exit 1; }
  f=$(ls -t /tmp/kt_$wl.* | head -1)
  python tools/ktrace_show.py $f > $O/ktrace_$wl.txt
  cat $O/ktrace_$wl.txt
done
