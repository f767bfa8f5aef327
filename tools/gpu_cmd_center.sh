# LayerNorm mean folded into the packed weights: policy tests, then A/B of the
# actor (mlp_lab) and the fused collection loop (prl_lab) against a lab build (uncentred, or prev = HEAD).
set -o pipefail
OUT=gpurun_out/${1:-center}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_policy.py tests/test_gpu_policy_rollout.py > $OUT/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/mlp_lab.py --variants base,serial --rows 65536,262144 --compute f16x3 > $OUT/mlp_f16x3.jsonl 2>$OUT/mlp.err &&
timeout -k 10 200 python -u tools/mlp_lab.py --variants base,serial --rows 65536 --compute f32 > $OUT/mlp_f32.jsonl 2>>$OUT/mlp.err &&
timeout -k 10 200 python -u tools/prl_lab.py --variants base,serial --envs 65536 --compute f16x3 > $OUT/prl_f16x3.jsonl 2>$OUT/prl.err
rc=$?; tail -3 $OUT/tests.log; cat $OUT/*.jsonl; exit $rc
