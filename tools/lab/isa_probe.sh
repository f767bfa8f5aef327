#!/bin/bash
# Device assembly of ONE kernel instantiation of csrc/drone_step.hip (seconds,
# not the library's minutes), then its basic-block / loop counts.
#   tools/lab/isa_probe.sh OUT.s ['rollout_kernel<float, 0, true, true, false>(RolloutArgs, Soa<float>)'] [-Dflags...]
set -e
OUT=${1:?out.s}
K=${2:-"rollout_kernel<float, 0, true, true, false>(RolloutArgs, Soa<float>)"}
shift; [ $# -gt 0 ] && shift
cd "$(dirname "$0")/../../reinforcement-learning-101_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Wall -Ibuild -I../include \
  --offload-device-only -S "-DDD_ISA_PROBE=$K" "$@" -o "$OUT" csrc/drone_step.hip 2>&1 | grep -v "unused during compilation" || true
SYM=$(grep -o '^_ZN2dd[A-Za-z0-9_]*:' "$OUT" | head -1 | tr -d ':')
python3 ../tools/isa_blocks.py "$OUT" "$SYM" | head -4
grep -E "\.(num_vgpr|numbered_sgpr), " "$OUT" | grep "$SYM" | sed 's/.*\.\(num_vgpr\|numbered_sgpr\)/\1/'
grep -c "v_writelane\|v_readlane" "$OUT" | sed 's/^/lane spills (read+write): /'
