#!/bin/bash
# One launcher for GPU-box sessions (run through gpurun from the repo root):
#
#   bash tools/gpu.sh <tag> <step> [<step> ...]
#
# Steps run in the order given, each under its own time limit, and the first
# failure ends the session (a fault, abort or time-out starts nothing more on
# the GPU).  Output goes to gpurun_out/<tag>/.
#
#   tests      pytest -m gpu (PYTEST_K: a -k expression)
#   smoke      __graft_entry__.smoke()
#   bench20    the driver's line: bench.py --gpus 1 --steps 20 --warmup 5
#   bench      bench.py with its defaults (every extra point)
#   prof20     rocprofv3 --kernel-trace --stats of the driver's exact command (bench.py --gpus 1 --steps 20
#              --warmup 5) and the trace summary of its 20 timed config-3 launches (c3_k20_trace_summary.json)
#   prof       rocprofv3 kernel traces: config 3, the 16.8M HBM point, the extra points
#   pmc        FETCH_SIZE / WRITE_SIZE passes of the step kernel at 262,144 and 16.8M drones
#   sq         SQ instruction counters of the step / rollout kernels (tools/pmc_sq.sh)
#   lab        tools/kernel_lab.py (VARIANTS, ENVS, LABARGS)
#   roll       tools/rollout_lab.py (VARIANTS, ENVS, ROLLARGS e.g. --philox), appended to <tag>/roll.jsonl
#   sqroll     SQ counters of dd_rollout per lab variant (tools/pmc_rollout_ab.sh; ROLLARGS, ROLLSUFFIX)
#   roll5      config 5 only: rocprof kernel trace of bench.py's 161 dd_rollout launches (65,536 x 256) and the
#              rollout kernel's FETCH_SIZE / WRITE_SIZE passes (tools/prof_driver.py --what rollout)
#   c5clk      config 5: GRBM_GUI_ACTIVE / SQ cycles per dispatch (the DVFS clock of each launch)
#   mr         tools/multirank_check.py on 2 gloo ranks sharing GPU 0 (torchrun), output in <tag>/mr/
#   py:<file>  python <file> (LABARGS passed through), output in <tag>/<file stem>.log
set -o pipefail
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp

run_step() {
    case "$1" in
    tests)
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
            ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1; local rc=$?; tail -2 $OUT/pytest_gpu.log; return $rc ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; local rc=$?
        tail -1 $OUT/smoke.log; return $rc ;;
    bench20)
        timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_k20.json 2> $OUT/bench_k20.err \
            && cat $OUT/bench_k20.json ;;
    bench)
        timeout -k 10 600 python bench.py ${BENCHARGS} > $OUT/bench_default.json 2> $OUT/bench_default.err \
            && python3 tools/bench_summary.py $OUT/bench_default.json ;;
    prof20)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_k20 -o bench -f csv -- python3 bench.py \
            --gpus 1 --steps 20 --warmup 5 > $OUT/prof_k20_bench.json 2> $OUT/prof20.err || return 1
        python3 tools/trace_summary.py $OUT/prof_k20/bench_kernel_trace.csv --kernel "step_kernel<float, 0, true, 0>" \
            --grid 262144 --slice 8:28 > $OUT/c3_k20_trace_summary.json && cut -c1-300 $OUT/c3_k20_trace_summary.json ;;
    prof)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o bench -f csv -- python3 bench.py \
            --steps 2000 --warmup 200 --cpu-baseline 0 --hbm-point 0 --rollout-point 0 --no-extra-points \
            > $OUT/prof_c3_bench.json 2> $OUT/prof.err &&
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_16m -o bench -f csv -- python3 bench.py \
            --envs-per-gpu 16777216 --steps 200 --warmup 20 --cpu-baseline 0 --hbm-point 0 --rollout-point 0 \
            --no-extra-points > $OUT/prof_16m_bench.json 2>> $OUT/prof.err &&
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_extra -o bench -f csv -- python3 bench.py \
            --steps 200 --warmup 20 --cpu-baseline 0 --hbm-point 0 > $OUT/prof_extra_bench.json 2>> $OUT/prof.err ;;
    pmc)
        for N in 262144 16777216; do
            for C in FETCH_SIZE WRITE_SIZE; do
                timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex step_kernel -d $OUT/pmc_${C}_$N -o pmc \
                    -f csv -- python3 bench.py --envs-per-gpu $N --steps 50 --warmup 5 --graph-steps 0 \
                    --cpu-baseline 0 --hbm-point 0 --rollout-point 0 --no-extra-points > /dev/null 2>> $OUT/pmc.err \
                    || return 1
            done
        done ;;
    sq)
        bash tools/pmc_sq.sh $TAG/sq > $OUT/sq_step_counters.txt; local rc=$?; cat $OUT/sq_step_counters.txt; return $rc ;;
    roll5)
        # bench.py's rollout_point schedule: 1 + 120 warm launches, then the 40 it times (last 40 of 161)
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5 -o roll -f csv -- python3 tools/prof_driver.py \
            --what rollout --envs 65536 --frames 256 --reps 161 > /dev/null 2> $OUT/roll5.err || return 1
        python3 tools/trace_summary.py $OUT/prof_c5/roll_kernel_trace.csv --kernel rollout_kernel --last 40 \
            > $OUT/c5_trace_summary.json || return 1
        for C in FETCH_SIZE WRITE_SIZE; do
            timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex rollout_kernel -d $OUT/pmc_roll_$C -o pmc -f csv \
                -- python3 tools/prof_driver.py --what rollout --envs 65536 --frames 256 --reps 5 > /dev/null \
                2>> $OUT/roll5.err || return 1
        done ;;
    c5clk)
        # the effective shader clock per config-5 launch: GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH, DVFS)
        timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace \
            -d $OUT/c5clk -o roll -f csv -- python3 tools/prof_driver.py --what rollout --envs 65536 --frames 256 \
            --reps 161 > /dev/null 2> $OUT/c5clk.err || return 1
        python3 tools/trace_summary.py $OUT/c5clk/roll_counter_collection.csv --kernel rollout_kernel --last 40 \
            > $OUT/c5clk_summary.json ;;
    lab)
        timeout -k 10 600 python tools/kernel_lab.py --variants ${VARIANTS:-base} --envs ${ENVS:-262144,1048576,16777216} \
            ${LABARGS} > $OUT/lab.jsonl 2> $OUT/lab.err; local rc=$?; cat $OUT/lab.jsonl; tail -5 $OUT/lab.err; return $rc ;;
    sqroll)
        ( OUT2=$TAG/sqroll; LABARGS="${ROLLARGS}" TAGSUFFIX="${ROLLSUFFIX}" bash tools/pmc_rollout_ab.sh $OUT2 $(echo ${VARIANTS:-base} | tr , " ") ) ;;
    roll)
        timeout -k 10 600 python tools/rollout_lab.py --variants ${VARIANTS:-base} --envs ${ENVS:-65536,262144} \
            ${ROLLARGS} >> $OUT/roll.jsonl 2>> $OUT/roll.err; local rc=$?; cat $OUT/roll.jsonl; tail -3 $OUT/roll.err; return $rc ;;
    micro:*)
        local m=${1#micro:}
        timeout -k 10 300 tools/micro/$m > $OUT/$m.jsonl 2> $OUT/$m.err; local rc=$?; cat $OUT/$m.jsonl; return $rc ;;
    mr)
        timeout -k 10 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
            --master-port 29517 tools/multirank_check.py --backend gloo --out $OUT/mr > $OUT/mr.log 2>&1; local rc=$?
        tail -3 $OUT/mr.log; return $rc ;;
    py:*)
        local f=${1#py:}; local stem=$(basename ${f%.py})
        timeout -k 10 ${PYTIMEOUT:-600} python -u $f ${LABARGS} > $OUT/$stem.log 2>&1; local rc=$?
        tail -${PYTAIL:-20} $OUT/$stem.log; return $rc ;;
    *)
        echo "unknown step $1"; return 2 ;;
    esac
}

for step in "$@"; do
    echo "== $step"
    run_step "$step" || { echo "== step $step failed (rc=$?); stopping"; exit 1; }
done
echo "== done"
