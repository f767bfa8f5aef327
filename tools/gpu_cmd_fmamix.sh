# The split's residual by v_fma_mix_f32 (lab DD_MLP_FMAMIX): bit-equality with
# the base build, then an A/B of the actor and the fused collection loop.
set -o pipefail
OUT=gpurun_out/${1:-fmamix}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/mlp_equal_check.py base fmamix > $OUT/equal_base_fmamix.log 2>&1 &&
timeout -k 10 200 python -u tools/mlp_lab.py --variants base,fmamix --rows 65536,262144 --compute f16x3 > $OUT/mlp_f16x3.jsonl 2>$OUT/mlp.err &&
timeout -k 10 200 python -u tools/prl_lab.py --variants base,fmamix --envs 65536 --compute f16x3 > $OUT/prl_f16x3.jsonl 2>$OUT/prl.err
rc=$?; grep -c "equal$" $OUT/equal_base_fmamix.log; grep -v "equal$" $OUT/equal_base_fmamix.log | tail -n 3; cat $OUT/*.jsonl; exit $rc
