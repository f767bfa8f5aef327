set -o pipefail
T=${1:-ab}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python tools/kernel_lab.py --variants ${VARIANTS:-prev,base} --envs ${ENVS:-262144,16777216} --rounds 15 --graph-steps 50 > gpurun_out/$T/klab.jsonl 2> gpurun_out/$T/klab.err &&
timeout -k 10 300 python tools/rollout_lab.py --variants ${VARIANTS:-prev,base} --envs 65536,262144 --rounds 9 > gpurun_out/$T/rlab.jsonl 2> gpurun_out/$T/rlab.err; rc=$?; cat gpurun_out/$T/klab.jsonl gpurun_out/$T/rlab.jsonl; tail -3 gpurun_out/$T/rlab.err; exit $rc
