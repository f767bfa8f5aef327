#!/bin/bash
# GPU box: SQ instruction / cycle counters of the config-3 step kernel for each
# lab build (tools/lab/step_eager.py, eager launches), one rocprofv3 --pmc pass
# per counter group and build, then per-wave averages of the last 40 launches.
#   bash tools/lab/sq_step_ab.sh TAG base noobs ...
set -o pipefail
OUT=gpurun_out/${1:?tag}
shift
mkdir -p $OUT
export TMPDIR=/tmp
groups=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS"
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"
)
for v in "$@"; do
  i=0
  for g in "${groups[@]}"; do
    timeout -s KILL 120 rocprofv3 --pmc $g --kernel-include-regex step_kernel -d $OUT/${v}_g$i -o pmc -f csv \
      -- python3 tools/lab/step_eager.py --variant $v --envs 262144 --steps 40 --warm 300 > /dev/null 2>> $OUT/err.log \
      || { echo "variant $v group $i failed"; exit 1; }
    i=$((i+1))
  done
done
python3 - "$OUT" "$@" <<'PY'
import csv, collections, json, os, sys
out, variants = sys.argv[1], sys.argv[2:]
for v in variants:
    row = {"variant": v}
    for i in range(2):
        f = os.path.join(out, f"{v}_g{i}", "pmc_counter_collection.csv")
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            if "step_kernel" in r["Kernel_Name"]:
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        last = [per[d] for d in sorted(per)][-40:]
        for k in last[0] if last else []:
            if k != "SQ_WAVES":
                row[k + "_per_wave"] = round(sum(x[k] / x["SQ_WAVES"] for x in last) / len(last), 1)
        row[f"launches_g{i}"] = len(last)
    print(json.dumps(row))
PY
