#!/bin/bash
# Fresh-box verification: GPU parity tests, smoke, default bench line.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
T=${1:-verify}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
tail -3 $OUT/pytest_gpu.log &&
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
cat $OUT/smoke.log &&
echo "== bench" && timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
cat $OUT/bench.json && echo "== done"
