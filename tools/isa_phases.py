#!/usr/bin/env python3
"""Where a kernel's instructions come from: the device assembly of a
translation unit built with line tables (-gline-tables-only), split by the
source function each instruction's innermost `.loc` falls in, then grouped
into the step's phases.  Static counts (every instruction once, rare paths
included); `--freq` weights each phase by how often a wave runs it
(tools/lab/branch_freq.py's per-wave rates) for an estimate of the dynamic
counts per wave.

    hipcc ... -gline-tables-only --offload-device-only -S -o /tmp/ds.s csrc/drone_step.hip
    python3 tools/isa_phases.py /tmp/ds.s '_ZN2dd11step_kernelIfLi0ELb1ELi0EEEvNS_8StepArgsENS_3SoaIT_EE'

Phases (by innermost source function; frame() split by its own sections):
  loads, thrust+physics, exact-flag tests, landing test, reward cascade,
  trig (fast sin / cos), speed / distance, re-spawn (Philox and draws),
  observation, stores, compaction + obs flush, exact redo (glibc restated),
  glue (the rest: finish_lane / step_tile control flow).
An instruction inlined from a system header (the HIP math wrappers) counts
to the last project source line before it.
"""
import argparse
import json
import os
import re
import sys
from collections import Counter, defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_blocks import classify  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "reinforcement-learning-101_amd", "csrc")

_DEF = re.compile(r"^\s*(?:template\s*<[^>]*>\s*)?(?:DD_HD\s+inline|__device__[\w\s]*?|inline|static)\s+[\w:<>,\s\*&]+?\b(\w+)\s*\(")


def functions_of(path):
    """[(first_line, name)] of the function definitions in a source file."""
    out = []
    for i, line in enumerate(open(path), 1):
        m = _DEF.match(line)
        if m and not line.rstrip().endswith(";"):
            out.append((i, m.group(1)))
    return out


def frame_sections(path):
    """Line ranges inside frame() (frame.h) by the comments that open them."""
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines, 1) if re.search(r"double frame\(const Consts", l))
    marks = {"exactness": None, "landing": None, "reward": None}
    for i in range(start, len(lines)):
        l = lines[i - 1]
        if marks["exactness"] is None and l.strip().startswith("// Exactness."):
            marks["exactness"] = i
        if marks["landing"] is None and "speed (get_speed), distance" in l:
            marks["landing"] = i
        if marks["reward"] is None and marks["landing"] and re.search(r"reward|_calculate_reward", l) and \
                l.strip().startswith("//") and i > marks["landing"] + 20:
            marks["reward"] = i
        if l.startswith("}") and i > start:
            end = i
            break
    return start, marks, end


PHASE_OF_FUNC = {
    "load_raw": "loads", "load_action": "loads", "at": "loads",
    "sincos_deg": "trig", "sincos_upright_deg": "trig", "hstep_c": "trig", "reduce_deg": "trig",
    "measure": "speed / distance", "sqrt_unscaled": "speed / distance",
    "spawn": "re-spawn", "spawn_from": "re-spawn", "spawn_words": "re-spawn", "draw_range": "re-spawn",
    "philox4x32_r": "re-spawn", "philox4x32_7": "re-spawn", "philox4x32_10": "re-spawn", "mulhilo": "re-spawn",
    "observe": "observation", "observe_values": "observation", "write_obs_row": "observation",
    "flush_obs_wave": "compaction + obs flush",
    "store_dynamics": "stores", "put_state": "stores", "put_out": "stores", "store_nt": "stores",
    "wrap_angle": "thrust+physics", "normalize_angle": "thrust+physics",
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("asm")
    p.add_argument("symbol")
    p.add_argument("--freq", help="JSON of per-wave rates {phase: rate} for the dynamic estimate")
    a = p.parse_args()
    lines = open(a.asm).read().split("\n")
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[int(m.group(1))] = os.path.basename(m.group(3) or m.group(2))
    funcs = {f: functions_of(os.path.join(CSRC, f)) for f in set(files.values()) if os.path.exists(os.path.join(CSRC, f))}
    fstart, fmarks, fend = frame_sections(os.path.join(CSRC, "frame.h"))
    libm = {"libm_ref.h", "libm_tables.h"}

    def func_at(fname, line):
        best = None
        for first, name in funcs.get(fname, []):
            if first <= line:
                best = name
        return best

    def phase(fname, line):
        if fname in libm:
            return "exact redo"
        if fname == "frame.h" and fstart <= line <= fend:
            if fmarks["reward"] and line >= fmarks["reward"]:
                return "reward cascade"
            if fmarks["landing"] and line >= fmarks["landing"]:
                return "landing test"
            if fmarks["exactness"] and line >= fmarks["exactness"]:
                return "exact-flag tests"
            return "thrust+physics"
        if fname == "trig.h":
            return PHASE_OF_FUNC.get(func_at(fname, line), "trig")
        if fname == "philox.h":
            return "re-spawn"
        name = func_at(fname, line)
        return PHASE_OF_FUNC.get(name, "glue")

    start = next(i for i, l in enumerate(lines) if l.startswith(a.symbol + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    cur = ("?", 0)
    counts = defaultdict(Counter)
    for l in lines[start:end]:
        s = l.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            loc = (files.get(int(m.group(1)), "?"), int(m.group(2)))
            # a system header's line (fabs, fma, sqrt ... inlined from the HIP
            # math headers): line tables name only the innermost inlined
            # function, so keep the last project line before it
            if loc[0] in funcs or loc[0] in libm:
                cur = loc
            continue
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        counts[phase(*cur)][classify(op)] += 1
    out = {"asm": a.asm, "symbol": a.symbol, "static": {ph: dict(c) for ph, c in sorted(counts.items())}}
    tot = Counter()
    for c in counts.values():
        tot.update(c)
    out["static_total"] = dict(tot)
    if a.freq:
        freq = json.load(open(a.freq))
        dyn = {ph: {k: round(v * freq.get(ph, 1.0), 1) for k, v in c.items()} for ph, c in counts.items()}
        out["dynamic_estimate_per_wave"] = dyn
        out["weights"] = freq
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
