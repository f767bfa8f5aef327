# Generic A/B call: rollout lab and/or step-kernel lab over $VARIANTS (lab builds from tools/build_variants.sh).
set -o pipefail
T=${1:-lab}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
if [ -n "$RENVS" ]; then
  timeout -k 10 600 python -u tools/rollout_lab.py --variants $VARIANTS --envs $RENVS --rounds ${ROUNDS:-7} > gpurun_out/$T/rlab.jsonl 2> gpurun_out/$T/rlab.err; rc=$?; cat gpurun_out/$T/rlab.jsonl; tail -3 gpurun_out/$T/rlab.err; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$KENVS" ]; then
  timeout -k 10 600 python -u tools/kernel_lab.py --variants $VARIANTS --envs $KENVS --rounds ${ROUNDS:-9} > gpurun_out/$T/klab.jsonl 2> gpurun_out/$T/klab.err; rc=$?; cat gpurun_out/$T/klab.jsonl; tail -3 gpurun_out/$T/klab.err; [ $rc -eq 0 ] || exit $rc
fi
