# A/B of the trie walk variants on the C3 encode: "K:WPE" (GBPE_WALK_SEG = K lanes per chunk, 0 = v5;
# GBPE_WALK_SEG_WPE = waves-per-EU hint); tokens vs fixture + kernel ms
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${WV:-0:0 4:0 4:6 4:8}; do
  k=${v%%:*}; e=${v#*:}
  GBPE_WALK_SEG=$k GBPE_WALK_SEG_WPE=$e timeout -k 10 400 python bench.py --no-cpu --no-c2 --no-c4 --no-c5 --steps 1 --warmup 0 --no-kernel-timing > gpurun_out/r3_walk$k.$e.json 2> gpurun_out/r3_walk$k.$e.err
  python - $k $e <<'PY' >> gpurun_out/r3_walk_ab.txt
import json, sys
l = [x for x in open(f"gpurun_out/r3_walk{sys.argv[1]}.{sys.argv[2]}.json") if x.startswith("{")][-1]
t = json.loads(l)["tokenize"]
print("WALK_SEG", sys.argv[1], "WPE", sys.argv[2], "equal", t.get("fixture_tokens_equal"), "walk %.3f scan %.3f compact %.3f ms" % (t["ms_walk"], t["ms_scan"], t["ms_compact"]), "kernels GB/s", t["gbps_kernels"], "e2e", t["gbps_end_to_end"])
PY
done
