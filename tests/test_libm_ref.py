"""CPU: libm_ref.h (the device restatement of glibc's pow(x, 2), sin, cos and
a fused sincos, used by the step's rare exact frames) equals this image's
glibc bit for bit: tools/check_libm_ref.cpp built against the committed
tables (csrc/libm_tables.h), on 4 M pow and ~1.2 M sin / cos inputs (random
over the frame's ranges, any finite magnitude for pow, the tiny and
range-boundary arguments); and the committed tables equal what
tools/gen_libm_tables.py reads out of this host's glibc 2.35 libm.so.6."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLES = os.path.join(REPO, "reinforcement-learning-101_amd", "csrc", "libm_tables.h")


def _glibc():
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    libc.gnu_get_libc_version.restype = ctypes.c_char_p
    return libc.gnu_get_libc_version().decode()


def test_committed_tables_are_this_glibcs():
    if _glibc() != "2.35":
        pytest.skip(f"host glibc {_glibc()}: the committed tables are glibc 2.35's (the reference's host)")
    r = subprocess.run(["python3", os.path.join(REPO, "tools", "gen_libm_tables.py"), "--check", TABLES],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_gen_refuses_other_glibc_and_missing_mpmath(tmp_path, monkeypatch):
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen", os.path.join(REPO, "tools", "gen_libm_tables.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    monkeypatch.setattr(gen, "glibc_version", lambda: "2.39")
    monkeypatch.setattr("sys.argv", ["gen", str(tmp_path / "t.h")])
    with pytest.raises(SystemExit, match="glibc 2.39"):
        gen.main()
    assert not (tmp_path / "t.h").exists()


def test_libm_ref_matches_glibc(tmp_path):
    if _glibc() != "2.35":
        pytest.skip(f"host glibc {_glibc()}: libm_ref.h restates 2.35")
    exe = tmp_path / "check_libm_ref"
    subprocess.run(["g++", "-O2", "-std=c++17", "-fno-builtin", "-ffp-contract=off",
                    f"-I{os.path.join(REPO, 'reinforcement-learning-101_amd', 'csrc')}",
                    os.path.join(REPO, "tools", "check_libm_ref.cpp"), "-o", str(exe), "-lm"], check=True)
    out = subprocess.run([str(exe), "1"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:]
    assert "0 / 4000015 differ" in out.stdout and "sin: 0 /" in out.stdout, out.stdout
