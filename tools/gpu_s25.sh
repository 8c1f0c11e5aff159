# Session-25 diagnostic (one GPU call): per-step times and phase stamps of the
# 1 GiB run with the round-5 grid (ktrace build).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s25
mkdir -p $O
GBPE_LIB=$PWD/gpu-bpe_amd/lib/kt/libgpubpe.so GBPE_KTRACE_OUT=/tmp/kt_en1g timeout -k 10 300 python -u tools/explore_1g.py en1g > $O/kt_en1g.log 2>&1 || { echo KTFAIL; tail -20 $O/kt_en1g.log; exit 1; }
f=$(ls -t /tmp/kt_en1g.* | head -1)
python tools/ktrace_show.py $f > $O/ktrace_en1g.txt
cat $O/ktrace_en1g.txt
python3 - <<'PY'
import json
for l in open("gpurun_out/s25/kt_en1g.log"):
    if l.startswith("{"):
        d = json.loads(l); s = d["step_ms_by_32"]
        print("loop", d["loop_s"], "first10", d["step_ms_first10"])
        print("by32", [round(x) for x in s], "cum", [round(sum(s[:i])) for i in (1, 2, 4, 8, len(s))])
PY
