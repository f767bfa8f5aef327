set -o pipefail
T=${1:-klab}
mkdir -p gpurun_out/$T
timeout -k 10 600 python tools/kernel_lab.py --variants ${VARIANTS} --envs ${ENVS:-262144,16777216} --rounds ${ROUNDS:-9} > gpurun_out/$T/lab.jsonl 2> gpurun_out/$T/lab.err; rc=$?; cat gpurun_out/$T/lab.jsonl; tail -3 gpurun_out/$T/lab.err; exit $rc
