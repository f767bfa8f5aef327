"""Source lint for a ROCm 7.2 clang miscompile that no compiler flag avoids.

`__builtin_bit_cast(T, v[i])` (or `v.x`) on an ext_vector ELEMENT bit-casts the
vector's first element whatever the index: clang takes the element's address
as the vector's.  E.g. with `u32x4 q` loaded from memory,
`__builtin_bit_cast(float, q[3])` stores `q[0]` (hipcc 7.2.26015, gfx950;
`global_load_dwordx4 v[2:5] ... global_store_dword v0, v2`).  The split
rollout's frame hand-over hit it.  This test rejects the
pattern in every device source; elements go through `__uint_as_float`,
`__float_as_uint` or a plain integer conversion instead.
"""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = [
    os.path.join(REPO, "reinforcement-learning-101_amd", "csrc"),
    os.path.join(REPO, "tools", "micro"),
]
VEC_TYPES = r"(?:f32x2|f32x4|f32x16|u32x4|u32x4_t|u64x2|f16x2|f16x8|D2x)"


def _device_files():
    for d in SOURCES:
        if not os.path.isdir(d):
            continue
        for name in sorted(os.listdir(d)):
            if name.endswith((".hip", ".h")):
                yield os.path.join(d, name)


def _bit_cast_operands(text):
    """Yield (line, operand) for every __builtin_bit_cast(T, operand)."""
    for m in re.finditer(r"__builtin_bit_cast\s*\(", text):
        i, depth, comma = m.end(), 1, None
        while i < len(text) and depth:
            c = text[i]
            if c in "([":
                depth += 1
            elif c in ")]":
                depth -= 1
            elif c == "," and depth == 1 and comma is None:
                comma = i
            i += 1
        if comma is not None:
            yield text.count("\n", 0, m.start()) + 1, text[comma + 1:i - 1].strip()


def find_element_bit_casts(text):
    vectors, arrays = set(), set()
    for m in re.finditer(VEC_TYPES + r"\s+(?:&\s*)?(\w+)\s*(\[)?", text):
        (arrays if m.group(2) else vectors).add(m.group(1))
    bad = []
    for line, op in _bit_cast_operands(text):
        if re.search(r"\.[xyzw]$", op) or re.search(r"\]\s*\[[^\]]*\]$", op):
            bad.append((line, op))
            continue
        m = re.fullmatch(r"(\w+)\s*\[[^\]]*\]", op)
        if m and m.group(1) in vectors and m.group(1) not in arrays:
            bad.append((line, op))
    return bad


def test_lint_catches_the_pattern():
    src = "u32x4 q = g[i];\nfloat r = __builtin_bit_cast(float, q[3]);\n" \
          "u32x4 w[6];\nuint32_t s = __builtin_bit_cast(uint32_t, w[5][2]);\n" \
          "f32x4 v;\nuint32_t t = __builtin_bit_cast(uint32_t, v.y);\n" \
          "f16x8 ok = __builtin_bit_cast(f16x8, blk[lane]);\n"
    assert [l for l, _ in find_element_bit_casts(src)] == [2, 4, 6]


@pytest.mark.parametrize("path", list(_device_files()), ids=os.path.basename)
def test_no_bit_cast_of_vector_elements(path):
    with open(path) as f:
        bad = find_element_bit_casts(f.read())
    assert not bad, f"{os.path.basename(path)}: __builtin_bit_cast of a vector element (miscompiled): {bad}"


PRODUCT = os.path.join(REPO, "reinforcement-learning-101_amd", "csrc")


@pytest.mark.parametrize("path", [p for p in _device_files() if p.startswith(PRODUCT)], ids=os.path.basename)
def test_product_sources_carry_no_lab_switches(path):
    """lab code stays out of the product kernels.  Experiments are
    A/B builds of committed revisions (tools/build_rev.sh), not -D switches or
    environment reads compiled into the product sources."""
    with open(path) as f:
        text = f.read()
    assert not re.search(r"\bDD_EXP_\w*", text), "lab switch DD_EXP_* in a product source"
    assert "getenv" not in text, "environment-driven kernel choice in a product source"
