# SQ counters of dd_mlp_forward (f16x3, 65,536 rows) and dd_policy_rollout
# (f16x3, 65,536 drones x 64 frames) on the current tree: one rocprofv3 pass per
# counter group, each under its own time limit.
set -o pipefail
OUT=gpurun_out/${1:-sq_mlp}
mkdir -p $OUT
export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA"
G2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"
for what in mlp prl; do
  if [ $what = mlp ]; then RX=mlp_kernel; A="--what mlp --envs 65536 --compute f16x3 --reps 5"; else RX=policy_rollout_kernel; A="--what prl --envs 65536 --frames 64 --compute f16x3 --reps 3"; fi
  i=0
  for g in "$G1" "$G2"; do
    timeout -s KILL 90 rocprofv3 --pmc $g --kernel-include-regex $RX -d $OUT/${what}_g$i -o pmc -f csv -- python3 tools/prof_driver.py $A > /dev/null 2>> $OUT/err.log || { echo "$what group $i failed"; exit 1; }
    i=$((i+1))
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for d in sorted(glob.glob(os.path.join(out, "*_g*"))):
    tot = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(os.path.basename(d), {k: round(v / max(n[k], 1)) for k, v in sorted(tot.items())})
PY
