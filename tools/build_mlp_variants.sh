#!/bin/bash
# Timing-only builds of dd_mlp_forward for A/B runs (tools/lab/mlp_lab.py): the
# product's other objects (make first) linked with policy_mlp.hip built under
# one -D switch per variant; outputs go to _native/lab/lib_<name>.so.
#   VARIANTS="nopair pv2 pv8" bash tools/build_mlp_variants.sh
set -e
cd "$(dirname "$0")/../reinforcement-learning-101_amd"
OUT=delivery_drone_amd/_native/lab
OBJ=build/obj
mkdir -p $OUT build/lab
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -I../include -Ibuild -mllvm -disable-machine-licm"
build() {
  ( /opt/rocm/bin/hipcc $FLAGS "${@:2}" -c -o build/lab/policy_mlp_$1.o csrc/policy_mlp.hip &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/lib_$1.so $OBJ/drone_step.o build/lab/policy_mlp_$1.o \
      $OBJ/policy_rollout.o $OBJ/render.o $OBJ/build_info.o ) &
}
for v in ${VARIANTS:-base}; do
  case $v in
    base) build base ;;
    nopair) build nopair -DDD_MLP_PAIR=0 ;;
    nocompute) build nocompute -DDD_EXP_MLP_NOCOMPUTE ;;
    maxilp) build maxilp -mllvm -amdgpu-sched-strategy=max-ilp ;;
    maxocc) build maxocc -mllvm -amdgpu-sched-strategy=max-occupancy ;;
    itermin) build itermin -mllvm -amdgpu-sched-strategy=iterative-minreg ;;
    pv*) build $v -DDD_MLP_PAIR_VALU=${v#pv} ;;
    *) echo "unknown variant $v"; exit 2 ;;
  esac
done
wait
