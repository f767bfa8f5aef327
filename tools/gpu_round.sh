#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel traces
# (config 3 and the 16M HBM point), PMC traffic passes.  Every GPU step has
# its own time limit and the steps are chained with && so the first failure
# ends the script.
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== build" && python -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1 &&
echo "== pytest -m gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 &&
tail -3 $OUT/pytest_gpu.log &&
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
cat $OUT/smoke.log &&
echo "== bench" && timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
cat $OUT/bench.json &&
echo "== rocprofv3 kernel trace (config 3)" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o bench -f csv -- python3 bench.py --steps 2000 --warmup 200 --cpu-baseline 0 --hbm-point 0 --rollout-point 0 --no-extra-points > $OUT/prof_c3_bench.json 2> $OUT/prof.err &&
echo "== rocprofv3 kernel trace (16M)" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_16m -o bench -f csv -- python3 bench.py --envs-per-gpu 16777216 --steps 200 --warmup 20 --cpu-baseline 0 --hbm-point 0 --rollout-point 0 --no-extra-points > $OUT/prof_16m_bench.json 2>> $OUT/prof.err &&
echo "== rocprofv3 kernel trace (extra points)" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_extra -o bench -f csv -- python3 bench.py --steps 200 --warmup 20 --cpu-baseline 0 --hbm-point 0 > $OUT/prof_extra_bench.json 2>> $OUT/prof.err &&
echo "== pmc" && for N in 262144 16777216; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex step_kernel -d $OUT/pmc_${C}_$N -o pmc -f csv -- python3 bench.py --envs-per-gpu $N --steps 50 --warmup 5 --graph-steps 0 --cpu-baseline 0 --hbm-point 0 --rollout-point 0 --no-extra-points > /dev/null 2>> $OUT/pmc.err || exit 1;
  done;
done && echo "== done"
