# Round 2, call j: DD_MLP_F16X3 — GPU policy tests, then f32 vs f16x3 policy points.
set -o pipefail
OUT=gpurun_out/r02j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py -v --timeout 120 --timeout-method thread > $OUT/pytest_policy.log 2>&1; rc=$?; tail -30 $OUT/pytest_policy.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u - > $OUT/points.jsonl 2> $OUT/points.err <<'PY'
import json, torch, bench
dev = torch.device("cuda", 0)
for n in (65536, 262144):
    for c in ("f32", "f16x3"):
        print(json.dumps(bench.policy_point(n, 0, dev, c)), flush=True)
for c in ("f32", "f16x3"):
    print(json.dumps(bench.policy_rollout_point(65536, 64, 0, dev, c)), flush=True)
PY
rc=$?; cat $OUT/points.jsonl; tail -3 $OUT/points.err; exit $rc
