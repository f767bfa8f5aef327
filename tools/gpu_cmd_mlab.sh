set -o pipefail
T=${1:-mlab}
mkdir -p gpurun_out/$T
timeout -k 10 400 python tools/mlp_lab.py --variants ${VARIANTS} --rows ${ROWS:-65536,262144} > gpurun_out/$T/mlab.jsonl 2> gpurun_out/$T/mlab.err; rc=$?; cat gpurun_out/$T/mlab.jsonl; tail -3 gpurun_out/$T/mlab.err; exit $rc
