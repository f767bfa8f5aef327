# Round 2, call a: GPU tests, store-policy A/B lab, bench at the driver's K/W and at the default.
set -o pipefail
T=${1:-r02a}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$T/bench_k20.json 2> gpurun_out/$T/bench_k20.err || exit $?
cat gpurun_out/$T/bench_k20.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('k20', d['value'], d['ms_per_step'], d['gpu_ms_per_step'], d['roofline']['frac'])"
timeout -k 10 600 python -u tools/kernel_lab.py --variants ${VARIANTS:-prev,base,wts,wto,wtall,wtntall,wtsnto,empty,nomath} --envs ${ENVS:-262144,1048576,16777216} --rounds ${ROUNDS:-9} > gpurun_out/$T/lab.jsonl 2> gpurun_out/$T/lab.err; rc=$?; cat gpurun_out/$T/lab.jsonl; tail -3 gpurun_out/$T/lab.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit $?
cat gpurun_out/$T/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['ms_per_step'], d['gpu_ms_per_step'], d['roofline']['frac'])"
