# dd_policy_rollout and dd_mlp_forward A/B on prebuilt lab variants: VARIANTS (comma list), COMPUTE.
set -o pipefail
OUT=gpurun_out/${1:-plab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/prl_lab.py --variants ${VARIANTS} --compute ${COMPUTE:-f16x3} --envs ${ENVS:-65536} > $OUT/prl.jsonl 2> $OUT/prl.err || { tail -3 $OUT/prl.err; exit 1; }
cat $OUT/prl.jsonl
timeout -k 10 300 python tools/mlp_lab.py --variants ${VARIANTS} --compute ${COMPUTE:-f16x3} --rows ${ROWS:-65536,262144} > $OUT/mlp.jsonl 2> $OUT/mlp.err || { tail -3 $OUT/mlp.err; exit 1; }
cat $OUT/mlp.jsonl
