"""Emit build/build_info.cpp: dd_build_info() returns the ABI version, the
sha256 of the device ISA of the step translation unit (drone_step.hip) and of
the fused policy rollout, and of the step and rollout kernels' own function
bodies (step_kernel_isa, rollout_kernel_isa), so a counter summary can be tied
to the exact code it was measured on (bench.py compares the row's kernel hash
before reporting roofline.traffic / rollout_point.traffic)."""
import hashlib
import re
import sys


def digest(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for line in f:
            if line.lstrip().startswith((b";", b"//")):  # comments only; every instruction and directive counts
                continue
            h.update(line)
    return h.hexdigest()[:16]


_LABEL_NO = re.compile(rb"\.(LBB|LCPI|Lfunc_end|Ltmp)\d+")


def kernel_digest(path: str, prefix: bytes) -> str:
    """sha256 of the bodies of every function whose symbol starts with
    `prefix` (from its `sym:` label to its `.Lfunc_end` label), comments
    skipped: a change elsewhere in the translation unit leaves it alone, so
    a PMC row of one kernel stays valid across edits of the others.  Label
    numbers that count the functions before it (.LBB<f>_<b>, .Lfunc_end<f>,
    .Ltmp<k>, .LCPI<f>_<k>) are normalised for the same reason."""
    h = hashlib.sha256()
    inside = False
    with open(path, "rb") as f:
        for line in f:
            if not inside and line.startswith(prefix) and line.split(None, 1)[0].endswith(b":"):
                inside = True
            if inside:
                if line.lstrip().startswith((b";", b"//")):
                    continue
                h.update(_LABEL_NO.sub(rb".\1", line))
                if line.startswith(b".Lfunc_end"):
                    inside = False
    return h.hexdigest()[:16]


step_isa, rollout_isa = sys.argv[1], sys.argv[2]
info = (f";step_isa={digest(step_isa)};policy_rollout_isa={digest(rollout_isa)}"
        f";step_kernel_isa={kernel_digest(step_isa, b'_ZN2dd11step_kernel')}"
        f";rollout_kernel_isa={kernel_digest(step_isa, b'_ZN2dd14rollout_kernel')}")
print('#include "dronestep.h"')
print("#define DD_STR2(x) #x")
print("#define DD_STR(x) DD_STR2(x)")
print(f'extern "C" const char* dd_build_info(void) {{ return "abi=" DD_STR(DD_ABI_VERSION) "{info}"; }}')
