#!/bin/bash
# Lab build: libdronestep with csrc/drone_step.hip's device code passed
# through tools/isa_post.py (device .s -> post-pass -> assemble -> link ->
# bundle -> host compile with the bundle embedded), the other sources as
# the Makefile builds them.  Output: delivery_drone_amd/_native/lab/lib_<name>.so
#   tools/build_post.sh <name> [extra hipcc flags]
set -e
NAME=${1:?name}
shift
cd "$(dirname "$0")/../reinforcement-learning-101_amd"
LLVM=/opt/rocm/lib/llvm/bin
OUT=delivery_drone_amd/_native/lab
T=build/post_$NAME
mkdir -p $OUT $T
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -I../include -Ibuild $*"
/opt/rocm/bin/hipcc $F --offload-device-only -S -o $T/drone_step.s csrc/drone_step.hip 2>&1 | grep -v "unused during compilation" || true
python3 ../tools/isa_post.py $T/drone_step.s $T/drone_step.post.s
$LLVM/clang -cc1as -triple amdgcn-amd-amdhsa -target-cpu gfx950 -filetype obj -o $T/drone_step.dev.o $T/drone_step.post.s
$LLVM/lld -flavor gnu -m elf64_amdgpu --no-undefined -shared -o $T/drone_step.hsaco $T/drone_step.dev.o
$LLVM/clang-offload-bundler -type=o -bundle-align=4096 \
  -targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--gfx950 \
  -input=/dev/null -input=$T/drone_step.hsaco -output=$T/drone_step.hipfb
/opt/rocm/bin/hipcc $F --cuda-host-only -Xclang -fcuda-include-gpubinary -Xclang $T/drone_step.hipfb \
  -c -o $T/drone_step.o csrc/drone_step.hip
/opt/rocm/bin/hipcc $F -mllvm -disable-machine-licm -c -o $T/policy_mlp.o csrc/policy_mlp.hip &
/opt/rocm/bin/hipcc $F -mllvm -disable-machine-licm -c -o $T/policy_rollout.o csrc/policy_rollout.hip &
/opt/rocm/bin/hipcc $F -c -o $T/render.o csrc/render.hip &
wait
/opt/rocm/bin/hipcc $F -shared -o $OUT/lib_$NAME.so $T/drone_step.o $T/policy_mlp.o $T/policy_rollout.o \
  $T/render.o build/obj/build_info.o
ls -la $OUT/lib_$NAME.so
