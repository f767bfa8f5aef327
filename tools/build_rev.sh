#!/bin/bash
# A lab build of the kernels as committed at git revision REV, against the
# current include/dronestep.h (older sources ignore the header's newer
# fields), into _native/lab/lib_NAME.so, for A/B runs of a past kernel
# against the working tree (tools/kernel_lab.py --variants NAME,base).
#   tools/build_rev.sh REV NAME
set -e
REV=${1:?rev}; NAME=${2:?name}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=/tmp/dd_rev_$NAME
rm -rf $SRC && mkdir -p $SRC
for f in $(git -C $ROOT ls-tree --name-only $REV reinforcement-learning-101_amd/csrc/); do
  git -C $ROOT show "$REV:$f" > $SRC/$(basename $f)
done
# before round 4 the glibc tables were generated into build/ (same data)
[ -f $SRC/libm_tables.h ] || cp $ROOT/reinforcement-learning-101_amd/csrc/libm_tables.h $SRC/
OUT=$ROOT/reinforcement-learning-101_amd/delivery_drone_amd/_native/lab
mkdir -p $OUT
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -I$ROOT/include -I$SRC"
pids=()
for s in drone_step policy_mlp policy_rollout render; do
  extra=""
  case $s in policy_mlp|policy_rollout) extra="-mllvm -disable-machine-licm";; esac
  /opt/rocm/bin/hipcc $FLAGS $extra -c -o $SRC/$s.o $SRC/$s.hip &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/lib_$NAME.so $SRC/*.o
echo "built $OUT/lib_$NAME.so from $REV"
