# Round 2, call b: GPU tests (notebook rollout added), short-region overheads by sync mode.
set -o pipefail
T=${1:-r02b}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for m in "" spin yield blocking; do
  DD_SYNC=$m timeout -k 10 180 python -u tools/k20_lab.py >> gpurun_out/$T/k20.jsonl 2>> gpurun_out/$T/k20.err || exit $?
done
cat gpurun_out/$T/k20.jsonl
