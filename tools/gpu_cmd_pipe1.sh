# Layer 1's split in the shadow of layer 2's cross terms (lab DD_MLP_PIPE1, since removed): the
# A/B of the actor (base / serial / pipe1), then bit-equality of the schedules.
set -o pipefail
OUT=gpurun_out/${1:-pipe1}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/mlp_lab.py --variants base,serial,pipe1 --rows 65536,262144 --compute f16x3 > $OUT/mlp_f16x3.jsonl 2>$OUT/mlp.err &&
timeout -k 10 200 python -u tools/mlp_lab.py --variants base,serial,pipe1 --rows 65536 --compute f32 > $OUT/mlp_f32.jsonl 2>>$OUT/mlp.err &&
timeout -k 10 200 python -u tools/mlp_equal_check.py serial pipe1 > $OUT/equal_serial_pipe1.log 2>&1 &&
timeout -k 10 200 python -u tools/mlp_equal_check.py serial base > $OUT/equal_serial_base.log 2>&1
rc=$?; cat $OUT/*.jsonl; for f in $OUT/equal_*.log; do tail -n 2 $f; done; exit $rc
