# Round 2, call e: fresh-container verification of HEAD (prebuilt in-tree library):
# GPU parity tests, smoke, the driver's bench command, the default bench line.
set -o pipefail
T=${1:-r02e}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && tail -3 $OUT/pytest_gpu.log &&
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log &&
echo "== bench K=20" && timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_k20.json 2> $OUT/bench_k20.err && head -c 700 $OUT/bench_k20.json && echo &&
echo "== bench default" && timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && head -c 700 $OUT/bench.json && echo
