# Round 2, call g: K=20/W=5 bench, extra points before vs after the headline (ABAB...).
set -o pipefail
OUT=gpurun_out/r02g
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $OUT/first_$i.json 2>> $OUT/err.log || exit 1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --points-after > $OUT/after_$i.json 2>> $OUT/err.log || exit 1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r02g/*.json")):
    d = json.load(open(f))
    print(f, d["value"], d["ms_per_step"], d["gpu_ms_per_step"])
PY
