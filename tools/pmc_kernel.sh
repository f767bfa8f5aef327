#!/bin/bash
# GPU box: SQ counters of one kernel family (tools/prof_driver.py --what W),
# one rocprofv3 pass per counter group, then a per-wave summary.
#   WHAT=rollout|step|mlp  ENVS=...  REGEX=kernel-name regex  LIB=alt .so (optional)
#   COMPUTE=f32|f16x3 (mlp)  EXTRA_GROUPS="A B;C D" more counter passes
set -o pipefail
OUT=gpurun_out/${1:-pmc_kernel}
WHAT=${WHAT:-rollout}; ENVS=${ENVS:-65536}; REGEX=${REGEX:-rollout_kernel}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
have() { grep -qw "$1" $OUT/counters.txt; }
groups=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS"
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"
 "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT"
 "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM"
)
[ -n "$EXTRA_GROUPS" ] && IFS=';' read -ra xg <<< "$EXTRA_GROUPS" && groups+=("${xg[@]}")
LIBARG=""; [ -n "$LIB" ] && LIBARG="--lib $LIB"
[ -n "$COMPUTE" ] && LIBARG="$LIBARG --compute $COMPUTE"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace -f csv -- python3 tools/prof_driver.py --what $WHAT --envs $ENVS $LIBARG > /dev/null 2>> $OUT/err.log || { echo "trace failed"; exit 1; }
i=0
for g in "${groups[@]}"; do
  sel=""; for c in $g; do have $c && sel="$sel $c"; done
  [ -z "$sel" ] && continue
  timeout -k 10 300 rocprofv3 --pmc $sel --kernel-include-regex $REGEX -d $OUT/g$i -o pmc -f csv -- python3 tools/prof_driver.py --what $WHAT --envs $ENVS --reps 3 $LIBARG > /dev/null 2>> $OUT/err.log || { echo "group $i failed"; exit 1; }
  i=$((i+1))
done
python3 - "$OUT" "$REGEX" <<'PY'
import csv, glob, os, re, sys, collections
out, rx = sys.argv[1], re.compile(sys.argv[2])
for f in sorted(glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        print("stats", r["Name"][:90], "calls", r["Calls"], "avg_ns", r["AverageNs"])
acc = collections.defaultdict(list)
for d in sorted(glob.glob(os.path.join(out, "g*"))):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if rx.search(r["Kernel_Name"]):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
waves = sum(acc.get("SQ_WAVES", [1])) / max(1, len(acc.get("SQ_WAVES", [1])))
for k, v in sorted(acc.items()):
    m = sum(v) / len(v)
    print(f"{k:28s} {m:16.1f}  per-wave {m / waves:10.2f}")
PY
