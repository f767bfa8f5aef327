#!/usr/bin/env python
"""Scan device assembly for the div_exact miscompile seen on ROCm 7.2 /
gfx950: `q0 = x * inv` written over x's register, then `fma(-q0, d, x)`
reading that register as x, i.e. `v_fma_f64 D, (-)A, B, A`.  The frame code
never forms fma(a, b, a), so any hit is the miscompile.
    python tools/scan_isa.py /tmp/isa/drone_step.s"""
import re
import sys


def scan(path):
    fn, hits = None, []
    for i, line in enumerate(open(path)):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            fn = m.group(1)
        m = re.match(r"\s*v_fma_f64 (v\[\d+:\d+\]), -?(v\[\d+:\d+\]), (\S+), (v\[\d+:\d+\])", line)
        if m and m.group(2) == m.group(4):
            hits.append((fn, i + 1, line.strip()))
    return hits


if __name__ == "__main__":
    hits = scan(sys.argv[1])
    for fn, ln, l in hits:
        print(f"{ln}: {fn[:70]}  {l}")
    sys.exit(1 if hits else 0)
