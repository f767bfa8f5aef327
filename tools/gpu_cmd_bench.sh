set -o pipefail
T=${1:-bench}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] &&
timeout -k 10 600 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err; rc=$?; cat gpurun_out/$T/bench.json; tail -3 gpurun_out/$T/bench.err; [ $rc -eq 0 ] &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 200 --warmup 20 --dist-backend gloo > gpurun_out/$T/bench_g2.json 2> gpurun_out/$T/bench_g2.err; rc=$?; cat gpurun_out/$T/bench_g2.json; tail -3 gpurun_out/$T/bench_g2.err; exit $rc
