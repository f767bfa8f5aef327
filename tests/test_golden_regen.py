"""CPU: every committed fixture under tests/golden/ regenerates byte for byte
from the reference (tests/golden/make_golden.py --out), so the parity anchors
are reproducible — the round-4 policy.npz was not (its reset spawns came from
numpy's unseeded global RNG).  Skipped where the reference checkout is absent
(the GPU box)."""
import filecmp
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
REF = os.environ.get("RL101_REFERENCE", "/root/reference")


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "delivery_drone", "game")),
                    reason="reference checkout absent")
def test_every_fixture_regenerates_byte_identically(tmp_path):
    subprocess.run([sys.executable, "-B", os.path.join(GOLDEN, "make_golden.py"), "--out", str(tmp_path)],
                   check=True, capture_output=True, timeout=600)
    made = sorted(os.listdir(tmp_path))
    committed = sorted(f for f in os.listdir(GOLDEN) if f.endswith((".npz", ".json")))
    assert made == committed
    differ = [f for f in made if not filecmp.cmp(tmp_path / f, os.path.join(GOLDEN, f), shallow=False)]
    assert not differ, differ
