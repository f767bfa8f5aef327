#!/bin/bash
# GPU box: list the gfx950 counters, then collect SQ/TA counters of the step
# kernel at two batch sizes (one rocprofv3 pass per counter group).
set -o pipefail
OUT=gpurun_out/${1:-pmc_sq}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
have() { grep -qw "$1" $OUT/counters.txt; }
groups=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS"
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"
 "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT"
 "GRBM_GUI_ACTIVE GRBM_COUNT"
 "TCC_HIT_sum TCC_MISS_sum"
)
i=0
for g in "${groups[@]}"; do
  sel=""; for c in $g; do have $c && sel="$sel $c"; done
  [ -z "$sel" ] && continue
  for N in 262144 16777216; do
    S=$(( N > 1000000 ? 20 : 50 ))
    timeout -k 10 300 rocprofv3 --pmc $sel --kernel-include-regex step_kernel -d $OUT/g${i}_$N -o pmc -f csv -- python3 bench.py --envs-per-gpu $N --steps $S --warmup 3 --graph-steps 0 --cpu-baseline 0 --hbm-point 0 --rollout-point 0 --no-extra-points > /dev/null 2>> $OUT/err.log || { echo "group $i N $N failed"; exit 1; }
  done
  i=$((i+1))
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for d in sorted(glob.glob(os.path.join(out, "g*_*"))):
    f = os.path.join(d, "pmc_counter_collection.csv")
    if not os.path.exists(f):
        continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "step_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(d), {k: round(sum(v) / len(v), 1) for k, v in acc.items()})
PY
