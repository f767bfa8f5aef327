set -o pipefail
OUT=gpurun_out/${1:-tests}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -25 $OUT/pytest_gpu.log; exit $rc
