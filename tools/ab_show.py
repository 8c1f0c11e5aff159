"""Print the headline fields of tools/ab_bench.sh results."""
import json
import sys

for name in sys.argv[1:]:
    j = json.loads(open(f"gpurun_out/ab_{name}.json").read().strip().splitlines()[-1])
    t = j["train_detail"]
    print(name, j["value"], j["roofline"]["frac"], {k: round(v, 1) if isinstance(v, float) else v
                                                  for k, v in t.items() if k.startswith("ms") or k == "sparse"})
