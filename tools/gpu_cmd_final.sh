# Final verification on a fresh box: GPU tests, smoke, the driver's K=20 bench line, the default bench line.
set -o pipefail
T=${1:-final}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
tail -2 $OUT/pytest_gpu.log &&
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
tail -1 $OUT/smoke.log &&
echo "== bench K=20" && timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_k20.json 2> $OUT/bench_k20.err &&
echo "== bench default" && timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err &&
python3 - $OUT <<'PY'
import json, sys
for f in ("bench_k20", "bench_default"):
    d = json.loads(open(f"{sys.argv[1]}/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"])
    if f == "bench_default":
        for k in ("policy_point_f16x3", "policy_rollout_point_f16x3", "policy_fused_point", "policy_fused_point_f16x3", "rollout_point"):
            v = d[k]; print(" ", k, v.get("us") or v.get("us_per_frame") or v.get("ms_per_rollout"), v.get("steps_per_s") or v.get("rows_per_s"))
PY
echo "== done"
