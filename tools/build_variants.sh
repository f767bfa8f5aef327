#!/bin/bash
# Timing-only builds of the step kernel for A/B runs (tools/kernel_lab.py).
# Each is the product source with one -D switch; outputs go to _native/lab/.
set -e
cd "$(dirname "$0")/../reinforcement-learning-101_amd"
OUT=delivery_drone_amd/_native/lab
mkdir -p $OUT
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -I../include"
build() { /opt/rocm/bin/hipcc $FLAGS "${@:2}" -o $OUT/lib_$1.so csrc/drone_step.hip & }
build base
build ocml -DDD_TRIG_OCML
build strided -DDD_OBS_STRIDED
build ntobs -DDD_NT_OBS
build w8 -DDD_STEP_MIN_WAVES=8
build w4 -DDD_STEP_MIN_WAVES=4
wait
ls -la $OUT
