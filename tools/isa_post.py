#!/usr/bin/env python3
"""Device-assembly post-pass for gfx950 (lab builds only, tools/build_post.sh:
the step / rollout kernels' .s rewritten before assembling them; measured and
dropped).

    python3 tools/isa_post.py IN.s OUT.s

Rewrites ``v_cndmask_b32_e32 vD, SRC0, vS1, vcc`` as the VOP3 form
``v_cndmask_b32_e64 vD, SRC0, vS1, vcc``: the same operation on the same
operands, 8 bytes instead of 4.  On gfx950 the VOP2 form costs a lone wave
(one wave per SIMD, as the config-5 rollout runs) about 3.5 issue slots
whenever VCC was not written by the instruction just before it, the VOP3
form about one (tools/micro/valu_cost.hip: a compare and the two selects of a
double, 7.3 vs 2.7 slots; profiles/r04/lab/valu_cost.jsonl).  The compiler
shrinks every select whose mask sits in VCC to the VOP2 form; this pass
undoes that.

Only forms the VOP3 encoding takes unchanged are rewritten: SRC0 a VGPR or
an inline constant (VOP3 has no literal on gfx9, and VCC already uses its one
scalar read).  Prints the counts; the output assembles to the same kernels
(descriptors, metadata and register counts untouched)."""
import re
import sys

INLINE_INT = {str(i) for i in range(-16, 65)}
INLINE_FLT = {"0.5", "-0.5", "1.0", "-1.0", "2.0", "-2.0", "4.0", "-4.0", "0.15915494"}
PAT = re.compile(r"^(\s*)v_cndmask_b32_e32(\s+)(v\d+), ([^,]+), (v\d+), vcc(\s*(?:;.*)?)$")


def src0_ok(s: str) -> bool:
    s = s.strip()
    return bool(re.fullmatch(r"v\d+", s)) or s in INLINE_INT or s in INLINE_FLT


def rewrite(lines):
    out, n, kept = [], 0, 0
    for line in lines:
        m = PAT.match(line)
        if m:
            ind, sp, d, s0, s1, tail = m.groups()
            if src0_ok(s0):
                line = f"{ind}v_cndmask_b32_e64{sp}{d}, {s0}, {s1}, vcc{tail}"
                n += 1
            else:
                kept += 1
        out.append(line)
    return out, n, kept


def main():
    src, dst = sys.argv[1], sys.argv[2]
    lines = open(src).read().split("\n")
    out, n, kept = rewrite(lines)
    with open(dst, "w") as f:
        f.write("\n".join(out))
    print(f"isa_post {src}: {n} v_cndmask_b32_e32 -> _e64, {kept} kept (literal / scalar src0)")


if __name__ == "__main__":
    main()
