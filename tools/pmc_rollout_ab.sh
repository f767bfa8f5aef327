#!/bin/bash
# GPU box: SQ instruction / cycle counters of dd_rollout (65,536 x 256) for
# each lab variant (tools/rollout_lab.py), one rocprofv3 pass per group.
#   [LABARGS=--philox] [TAGSUFFIX=_p] bash tools/pmc_rollout_ab.sh <outdir> <variant> [<variant> ...]
set -o pipefail
OUT=gpurun_out/${1:?out}
shift
mkdir -p $OUT
export TMPDIR=/tmp
groups=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM"
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"
)
for v in "$@"; do
  i=0
  for g in "${groups[@]}"; do
    timeout -s KILL 120 rocprofv3 --pmc $g --kernel-include-regex rollout_kernel -d $OUT/${v}${TAGSUFFIX}_g$i -o pmc -f csv -- \
      python3 tools/rollout_lab.py --variants $v --envs 65536 --rounds 2 ${LABARGS} > /dev/null 2>> $OUT/err.log \
      || { echo "variant $v group $i failed"; exit 1; }
    i=$((i+1))
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for d in sorted(glob.glob(os.path.join(out, "*_g*"))):
    f = os.path.join(d, "pmc_counter_collection.csv")
    if not os.path.exists(f):
        continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    # per wave-frame: 1,024 waves x 256 frames
    print(os.path.basename(d), {k: round(sum(v) / len(v) / (1024 * 256), 1) for k, v in acc.items()})
PY
