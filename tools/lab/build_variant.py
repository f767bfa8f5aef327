#!/usr/bin/env python
"""A lab build of the working tree with one source edit, for A/B runs
(tools/kernel_lab.py, tools/lab/mlp_lab.py, tools/lab/prl_lab.py): copies
reinforcement-learning-101_amd/csrc to /tmp, applies string replacements to
one source (each OLD must occur exactly once), compiles that source and links
it with the product's other objects into _native/lab/lib_NAME.so.  The
product sources stay free of lab switches.

    python tools/lab/build_variant.py NAME FILE OLD NEW [OLD NEW ...] [-- FILE2 OLD NEW ...]

Edits to several sources are groups separated by "--".  DD_VARIANT_UNITS
(comma list, e.g. drone_step) limits the rebuilt translation units; the
others are linked from the product build (a lab timing the step kernel need
not wait for policy_rollout.hip).
"""
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(REPO, "reinforcement-learning-101_amd")
UNITS = ("drone_step", "policy_mlp", "policy_rollout", "render", "device_memory")  # the Makefile's SRCS
FLAGS = {"policy_mlp": ["-mllvm", "-disable-machine-licm"], "policy_rollout": ["-mllvm", "-disable-machine-licm"]}


def main():
    name, rest = sys.argv[1], sys.argv[2:]
    groups, cur = [], []
    for a in rest:
        if a == "--":
            groups.append(cur)
            cur = []
        else:
            cur.append(a)
    groups.append(cur)
    src = f"/tmp/dd_variant_{name}"
    shutil.rmtree(src, ignore_errors=True)
    shutil.copytree(os.path.join(PKG, "csrc"), src)
    fnames = []
    for grp in groups:
        fname, edits = grp[0], grp[1:]
        fnames.append(fname)
        path = os.path.join(src, fname)
        text = open(path).read()
        for old, new in zip(edits[::2], edits[1::2]):
            if text.count(old) != 1:
                raise SystemExit(f"{fname}: {old!r} occurs {text.count(old)} times")
            text = text.replace(old, new)
        open(path, "w").write(text)
    # the translation units the edit lands in (a header: every unit that includes it)
    def includes(f, seen=None):
        seen = seen if seen is not None else set()
        for line in open(os.path.join(src, f)):
            if line.startswith('#include "'):
                inc = line.split('"')[1]
                if inc not in seen and os.path.exists(os.path.join(src, inc)):
                    seen.add(inc)
                    includes(inc, seen)
        return seen
    units = [u for u in UNITS
             if any(f == u + ".hip" or f in includes(u + ".hip") for f in fnames)]
    if os.environ.get("DD_VARIANT_UNITS"):
        units = [u for u in units if u in os.environ["DD_VARIANT_UNITS"].split(",")]
    objs = []
    for u in UNITS:
        if u in units:
            o = os.path.join(src, u + ".o")
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                            "-fPIC", f"-I{os.path.join(REPO, 'include')}", f"-I{src}", *FLAGS.get(u, []),
                            "-c", "-o", o, os.path.join(src, u + ".hip")], check=True)
        else:
            o = os.path.join(PKG, "build", "obj", u + ".o")
        objs.append(o)
    objs.append(os.path.join(PKG, "build", "obj", "build_info.o"))
    out = os.path.join(PKG, "delivery_drone_amd", "_native", "lab", f"lib_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o", out, *objs], check=True)
    print(f"built {out} ({', '.join(fnames)}; rebuilt {units})")


if __name__ == "__main__":
    main()
