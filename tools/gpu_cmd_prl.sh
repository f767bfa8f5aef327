# Fused policy rollout (dd_policy_rollout) vs the two-kernel hipGraph loop.
set -o pipefail
OUT=gpurun_out/${1:-prl}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u - > $OUT/points.jsonl 2> $OUT/points.err <<'PY'
import json, torch, bench
dev = torch.device("cuda", 0)
for n, frames in ((65536, 64), (65536, 256), (262144, 64)):
    for c in ("f32", "f16x3"):
        if frames == 64:
            print(json.dumps(bench.policy_rollout_point(n, frames, 0, dev, c)), flush=True)
        print(json.dumps(bench.policy_fused_point(n, frames, 0, dev, c)), flush=True)
PY
rc=$?; cat $OUT/points.jsonl; tail -3 $OUT/points.err; exit $rc
