"""Emit build/build_info.cpp: dd_build_info() returns the ABI version and the
sha256 of the device ISA of the step translation unit (drone_step.hip, the
kernels whose PMC traffic profiles/pmc_traffic.json records) and of the fused
policy rollout, so a counter summary can be tied to the exact code it was
measured on (bench.py compares them before reporting roofline.traffic)."""
import hashlib
import sys


def digest(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for line in f:
            if line.lstrip().startswith((b";", b"//")):  # comments only; every instruction and directive counts
                continue
            h.update(line)
    return h.hexdigest()[:16]


step_isa, rollout_isa = sys.argv[1], sys.argv[2]
info = f";step_isa={digest(step_isa)};policy_rollout_isa={digest(rollout_isa)}"
print('#include "dronestep.h"')
print("#define DD_STR2(x) #x")
print("#define DD_STR(x) DD_STR2(x)")
print(f'extern "C" const char* dd_build_info(void) {{ return "abi=" DD_STR(DD_ABI_VERSION) "{info}"; }}')
