#!/bin/bash
# One profiling session on a GPU box, from the prebuilt in-tree library:
# default bench line, rocprofv3 kernel traces (config 3, the 16.8M HBM point,
# the extra points) and PMC FETCH_SIZE / WRITE_SIZE passes of the step kernel.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== bench" && timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
cat $OUT/bench.json &&
echo "== rocprofv3 config 3" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o bench -f csv -- python3 bench.py --steps 2000 --warmup 200 --cpu-baseline 0 --hbm-point 0 --rollout-point 0 --no-extra-points > $OUT/prof_c3_bench.json 2> $OUT/prof.err &&
echo "== rocprofv3 16M" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_16m -o bench -f csv -- python3 bench.py --envs-per-gpu 16777216 --steps 200 --warmup 20 --cpu-baseline 0 --hbm-point 0 --rollout-point 0 --no-extra-points > $OUT/prof_16m_bench.json 2>> $OUT/prof.err &&
echo "== rocprofv3 extra points" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_extra -o bench -f csv -- python3 bench.py --steps 200 --warmup 20 --cpu-baseline 0 --hbm-point 0 > $OUT/prof_extra_bench.json 2>> $OUT/prof.err &&
echo "== pmc" && for N in 262144 16777216; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex step_kernel -d $OUT/pmc_${C}_$N -o pmc -f csv -- python3 bench.py --envs-per-gpu $N --steps 50 --warmup 5 --graph-steps 0 --cpu-baseline 0 --hbm-point 0 --rollout-point 0 --no-extra-points > /dev/null 2>> $OUT/pmc.err || exit 1;
  done;
done && echo "== done"
