# Round 2, call d: GPU tests with the split rollout kernel, rollout A/B (split on/off) by batch size.
set -o pipefail
T=${1:-r02d}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/rollout_lab.py --variants prev,splitoff,spliton --envs 65536,131072,262144 --rounds 7 > gpurun_out/$T/rlab.jsonl 2> gpurun_out/$T/rlab.err; rc=$?; cat gpurun_out/$T/rlab.jsonl; tail -3 gpurun_out/$T/rlab.err; exit $rc
