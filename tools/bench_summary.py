"""Print the headline and the extra points of a bench.py JSON line (GPU-box session summary)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms_per_step", d["ms_per_step"], "frac", d["roofline"]["frac"])
for k, v in d.items():
    if isinstance(v, dict) and "_point" in k:
        keys = ("us", "us_per_frame", "ms_per_rollout", "steps_per_s", "rows_per_s", "frac")
        print(" ", k, {q: v[q] for q in keys if q in v})
