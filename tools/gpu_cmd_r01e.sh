set -o pipefail
T=${1:-r01e}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -m pytest tests/test_gpu_rollout.py -x -q > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python tools/rollout_lab.py --variants prev,base,rnoact --envs 65536,262144 --rounds 9 > gpurun_out/$T/rlab.jsonl 2> gpurun_out/$T/rlab.err &&
timeout -k 10 300 python tools/rollout_lab.py --variants prev,base,rnoact --envs 65536 --rounds 9 --no-obs >> gpurun_out/$T/rlab.jsonl 2>> gpurun_out/$T/rlab.err; rc=$?; cat gpurun_out/$T/rlab.jsonl; tail -3 gpurun_out/$T/rlab.err; exit $rc
