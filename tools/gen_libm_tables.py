#!/usr/bin/env python3
"""Emit libm_tables.h: the data tables of the C library's pow, sin and cos,
read from the libm.so.6 of this image (glibc 2.35, x86_64), for the device
restatement of those functions in csrc/libm_ref.h.

Why: the reference computes its squares as Python / numpy ``v ** 2`` (glibc
``pow(v, 2.0)``, which differs from the correctly rounded ``v * v`` on ~0.09 %
of inputs) and its trigonometry as ``np.sin`` / ``np.cos`` (glibc ``sin`` /
``cos``).  The step kernel uses its own fast versions and, on the rare frame
whose predicates sit within a hair of a boundary, re-evaluates them with a
restatement of glibc's published algorithms so the done / landed / crashed
flags equal the reference's bit for bit.  The algorithms'
coefficient tables are data; they are taken from the installed library
rather than retyped, located by their published header constants and checked
against independently computed values before use:

* ``__pow_log_data`` (sysdeps/ieee754/dbl-64/e_pow_log_data.c): ln2hi, ln2lo,
  7 polynomial coefficients, 128 x {invc, pad, logc, logctail};
* ``__exp_data`` (e_exp_data.c): invln2N, shift, -ln2hi/N, -ln2lo/N, 4
  coefficients, exp2 data (unused), 256 table words;
* ``__sincostab`` (sincostab.c): 440 doubles, {sin, sin tail, cos, cos tail}
  of i/128 for i = 0..109.

    python3 tools/gen_libm_tables.py OUT.h [libm path]
    python3 tools/gen_libm_tables.py --check reinforcement-learning-101_amd/csrc/libm_tables.h

The product builds from the committed csrc/libm_tables.h (made by this
script on the glibc 2.35 image, so any build host gives the same bits); this
script regenerates or checks it.  It refuses to run against any glibc but
2.35 (libm_ref.h restates 2.35's algorithms, and the reference's bits are
those of the host that runs it, glibc 2.35 in this image) and without mpmath
(the sin / cos table check is not optional).  libm.so.6 is located the way
the dynamic linker finds it (ctypes loads it; its path is read from
/proc/self/maps), not at a fixed Debian path.
"""
import math
import os
import struct
import sys

from fractions import Fraction

GLIBC = "2.35"


def glibc_version() -> str:
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    libc.gnu_get_libc_version.restype = ctypes.c_char_p
    return libc.gnu_get_libc_version().decode()


def find_libm() -> str:
    """The libm.so.6 the dynamic linker loads for this process."""
    import ctypes
    ctypes.CDLL("libm.so.6")
    for line in open("/proc/self/maps"):
        parts = line.split()
        if len(parts) >= 6 and os.path.basename(parts[5]).startswith("libm.so"):
            return os.path.realpath(parts[5])
    raise SystemExit("gen_libm_tables: libm.so.6 is loaded but not in /proc/self/maps")


LIBM = None  # set in main()


def find_all(blob: bytes, pat: bytes):
    out, s = [], 0
    while True:
        k = blob.find(pat, s)
        if k < 0:
            return out
        out.append(k)
        s = k + 1


def doubles(blob, off, n):
    return list(struct.unpack_from(f"<{n}d", blob, off))


def words(blob, off, n):
    return list(struct.unpack_from(f"<{n}Q", blob, off))


def pow_log_data(blob):
    ln2hi, ln2lo = float.fromhex("0x1.62e42fefa3800p-1"), float.fromhex("0x1.ef35793c76730p-45")
    for k in find_all(blob, struct.pack("<2d", ln2hi, ln2lo)):
        poly = doubles(blob, k + 16, 7)
        tab = doubles(blob, k + 72, 4 * 128)
        if poly[0] != -0.5 or tab[0] != float.fromhex("0x1.6ap+0") or tab[1] != 0.0:
            continue  # log()'s table shares the header; pow's has A[0] = -0.5 exactly and invc[0] = 0x1.6ap0
        for i in range(128):  # invc is j/N or j/N/2, logc ~ -log(invc) to 2^-43
            invc, pad, logc, logctail = tab[4 * i:4 * i + 4]
            assert pad == 0.0 and 0.7 < invc < 1.42, (i, invc)
            assert abs(logc + math.log(invc)) < 1e-12, (i, logc)
            assert float(Fraction(invc) * 256).is_integer()
        return ln2hi, ln2lo, poly, tab
    raise SystemExit("pow log table not found in " + LIBM)


def exp_data(blob):
    head = struct.pack("<2d", float.fromhex("0x1.71547652b82fep7"), float.fromhex("0x1.8p52"))
    for k in find_all(blob, head):
        d = doubles(blob, k, 4)
        poly = doubles(blob, k + 32, 4)
        tab = words(blob, k + 14 * 8, 256)
        if tab[0] != 0 or tab[1] != 0x3FF0000000000000:
            continue
        for i in range(128):  # sbits + (i << 45) is 2^(i/128) rounded; tail is its relative remainder
            h = struct.unpack("<d", struct.pack("<Q", tab[2 * i + 1] + (i << 45)))[0]
            assert abs(h - 2.0 ** (i / 128)) <= 2 * math.ulp(h), i
            t = struct.unpack("<d", struct.pack("<Q", tab[2 * i]))[0]
            assert abs(t) < 2 ** -52, (i, t)
        return d, poly, tab
    raise SystemExit("exp table not found in " + LIBM)


def sincostab(blob):
    s1 = math.sin(1 / 128)
    for k in find_all(blob, struct.pack("<d", s1)):
        t = doubles(blob, k - 32, 440)
        if t[:4] != [0.0, 0.0, 1.0, 0.0]:
            continue
        try:
            import mpmath
        except ImportError:
            raise SystemExit("gen_libm_tables: mpmath is needed to check the sin / cos table")
        mpmath.mp.prec = 200
        for i in range(110):  # {sn, ssn, cs, ccs}: sin / cos of i/128 as double-double
            x = mpmath.mpf(i) / 128
            for j, f in ((0, mpmath.sin), (2, mpmath.cos)):
                hi, lo = t[4 * i + j], t[4 * i + j + 1]
                assert abs(mpmath.mpf(hi) + mpmath.mpf(lo) - f(x)) < mpmath.mpf(2) ** -100, (i, j)
        return t
    raise SystemExit("sincos table not found in " + LIBM)


def c_doubles(vals, per_line=4):
    items = [float.hex(v) for v in vals]
    return ",\n    ".join(", ".join(items[i:i + per_line]) for i in range(0, len(items), per_line))


def render(path: str) -> str:
    blob = open(path, "rb").read()
    ln2hi, ln2lo, lpoly, ltab = pow_log_data(blob)
    ed, epoly, etab = exp_data(blob)
    sct = sincostab(blob)
    lines = [
        "// Generated by tools/gen_libm_tables.py from glibc " + GLIBC + "'s libm.so.6 (x86_64) — do not edit.",
        "// Data tables of glibc's pow (e_pow_log_data.c, e_exp_data.c) and sin / cos",
        "// (sincostab.c) for csrc/libm_ref.h.  Numeric data of the GNU C Library",
        "// (LGPL-2.1-or-later); see THIRD_PARTY_NOTICES.md.",
        "#pragma once",
        "#define DD_LIBM_POW_LN2HI " + float.hex(ln2hi),
        "#define DD_LIBM_POW_LN2LO " + float.hex(ln2lo),
        "#define DD_LIBM_POW_POLY {" + ", ".join(float.hex(v) for v in lpoly) + "}",
        "#define DD_LIBM_POW_TAB {  /* invc, logc, logctail */ \\\n    " +
        c_doubles([v for i in range(128) for v in (ltab[4 * i], ltab[4 * i + 2], ltab[4 * i + 3])], 3)
        .replace("\n", " \\\n") + "}",
        "#define DD_LIBM_EXP_INVLN2N " + float.hex(ed[0]),
        "#define DD_LIBM_EXP_SHIFT " + float.hex(ed[1]),
        "#define DD_LIBM_EXP_NEGLN2HIN " + float.hex(ed[2]),
        "#define DD_LIBM_EXP_NEGLN2LON " + float.hex(ed[3]),
        "#define DD_LIBM_EXP_POLY {" + ", ".join(float.hex(v) for v in epoly) + "}",
        "#define DD_LIBM_EXP_TAB {  /* tail, sbits */ \\\n    " +
        ",\n    ".join(", ".join(f"0x{w:016x}ull" for w in etab[i:i + 4]) for i in range(0, 256, 4))
        .replace("\n", " \\\n") + "}",
        "#define DD_LIBM_SINCOS_TAB {  /* sn, ssn, cs, ccs of i/128 */ \\\n    " +
        c_doubles(sct, 4).replace("\n", " \\\n") + "}",
    ]
    return "\n".join(lines) + "\n"


def main():
    global LIBM
    args = [a for a in sys.argv[1:] if a != "--check"]
    check = "--check" in sys.argv[1:]
    if not args:
        raise SystemExit(__doc__)
    have = glibc_version()
    if have != GLIBC:
        raise SystemExit(f"gen_libm_tables: this host runs glibc {have}; libm_ref.h restates glibc {GLIBC}'s "
                         f"pow / sin / cos, so its tables must come from {GLIBC} (keep the committed "
                         f"csrc/libm_tables.h)")
    LIBM = os.path.realpath(args[1]) if len(args) > 1 else find_libm()
    text = render(LIBM)
    if check:
        same = open(args[0]).read() == text
        print(f"{args[0]}: {'equal to' if same else 'DIFFERS from'} the tables of {LIBM} (glibc {have})")
        raise SystemExit(0 if same else 1)
    with open(args[0], "w") as f:
        f.write(text)


if __name__ == "__main__":
    main()
