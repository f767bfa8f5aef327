# MLP A/B (tools/mlp_lab.py) for one compute mode: VARIANTS, COMPUTE, ROWS.
set -o pipefail
T=${1:-mlab}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python tools/mlp_lab.py --variants ${VARIANTS} --compute ${COMPUTE:-f16x3} --rows ${ROWS:-65536,262144} > gpurun_out/$T/lab.jsonl 2> gpurun_out/$T/lab.err; rc=$?; cat gpurun_out/$T/lab.jsonl; tail -3 gpurun_out/$T/lab.err; exit $rc
