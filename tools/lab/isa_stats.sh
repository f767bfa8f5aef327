#!/bin/bash
# Device assembly of drone_step.hip (+ extra -D flags) and the register /
# spill metadata of the step and rollout kernels (no GPU needed).
#   tools/lab/isa_stats.sh [-DFLAG ...]   -> /tmp/isa/drone_step.s
set -e
cd "$(dirname "$0")/../../reinforcement-learning-101_amd"
mkdir -p /tmp/isa
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -I../include \
  --offload-device-only -S -o /tmp/isa/drone_step.s "$@" csrc/drone_step.hip 2>&1 | grep -v "unused during compilation" || true
python3 - <<'PY'
import re
s = open("/tmp/isa/drone_step.s").read()
for m in re.finditer(r"\.name:\s+(\S+)\n(.*?)(?=\n  - |\Z)", s, re.S):
    name, body = m.group(1), m.group(2)
    if not re.search(r"(step|rollout)_kernelIfLi[03]ELb1E", name):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", body) or [None, "?"])[1]
    print(f"{name[:60]:60s} vgpr {g('vgpr_count'):>4} sgpr {g('sgpr_count'):>4} "
          f"sgpr_spill {g('sgpr_spill_count'):>3} vgpr_spill {g('vgpr_spill_count'):>3} lds {g('group_segment_fixed_size')}")
PY
