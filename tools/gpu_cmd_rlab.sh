set -o pipefail
T=${1:-rlab}
mkdir -p gpurun_out/$T
timeout -k 10 300 python tools/rollout_lab.py --variants ${VARIANTS} --envs ${ENVS:-65536,262144} --rounds 9 > gpurun_out/$T/rlab.jsonl 2> gpurun_out/$T/rlab.err &&
timeout -k 10 300 python tools/rollout_lab.py --variants ${VARIANTS} --envs 65536 --rounds 9 --no-obs >> gpurun_out/$T/rlab.jsonl 2>> gpurun_out/$T/rlab.err; rc=$?; cat gpurun_out/$T/rlab.jsonl; tail -3 gpurun_out/$T/rlab.err; exit $rc
