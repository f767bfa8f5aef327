# Timeline lab (tools/timeline_lab.py) on prebuilt lab variants: VARIANTS (comma list), ENVS.
set -o pipefail
T=${1:-tl}
mkdir -p gpurun_out/$T
timeout -k 10 400 python tools/timeline_lab.py --variants ${VARIANTS} --envs ${ENVS:-262144} --rounds ${ROUNDS:-8} > gpurun_out/$T/tl.jsonl 2> gpurun_out/$T/tl.err; rc=$?
python3 - gpurun_out/$T/tl.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["variant"], d["envs"], d["us_per_step_median"], d["us_per_step_min"], "span", d["span_us_median"], "out", d["outside_span_us"],
          "load", d["load_wait_us_pct"][2], "t2", d["t2_frame_done_pct"][2], d["t2_frame_done_pct"][4], "drain", d["store_drain_us_pct"][2])
PY
tail -3 gpurun_out/$T/tl.err; exit $rc
