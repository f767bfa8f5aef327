# Rolled Philox for rare draws (spawns, rollout action blocks): parity tests that
# cover spawns, then A/B of the step (kernel_lab) and the rollout (rollout_lab,
# tensor and in-kernel actions) against the HEAD build.
set -o pipefail
OUT=gpurun_out/${1:-rolled}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rollout.py tests/test_gpu_parity.py tests/test_gpu_notebook_rollout.py tests/test_gpu_policy_rollout.py > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/kernel_lab.py --variants base,prev --envs 262144,16777216 --rounds 9 > $OUT/step.jsonl 2>$OUT/step.err &&
timeout -k 10 300 python -u tools/rollout_lab.py --variants base,prev --envs 65536,262144 --philox --rounds 9 > $OUT/roll_philox.jsonl 2>$OUT/roll.err &&
timeout -k 10 300 python -u tools/rollout_lab.py --variants base,prev --envs 65536,262144 --rounds 9 > $OUT/roll_tensor.jsonl 2>>$OUT/roll.err
rc=$?; tail -2 $OUT/tests.log; cat $OUT/*.jsonl; exit $rc
