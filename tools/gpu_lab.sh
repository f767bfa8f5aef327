#!/bin/bash
# GPU box: correctness gate for the current build, then A/B kernel timings.
set -o pipefail
TAG=${1:-lab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] &&
timeout -k 10 600 python tools/kernel_lab.py --variants ${VARIANTS:-base} --envs ${ENVS:-262144,1048576,16777216} ${LABARGS:-} > $OUT/lab.jsonl 2> $OUT/lab.err; rc=$?; cat $OUT/lab.jsonl; tail -5 $OUT/lab.err; exit $rc
