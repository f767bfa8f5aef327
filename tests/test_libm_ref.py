"""CPU: libm_ref.h (the device restatement of glibc's pow(x, 2), sin, cos and
a fused sincos, used by the step's rare exact frames) equals this image's
glibc bit for bit: tools/check_libm_ref.cpp built against the tables
tools/gen_libm_tables.py reads out of libm.so.6, on 4 M pow and ~1.2 M
sin / cos inputs (random over the frame's ranges, any finite magnitude for
pow, the tiny and range-boundary arguments)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_libm_ref_matches_glibc(tmp_path):
    hdr = tmp_path / "libm_tables.h"
    subprocess.run(["python3", os.path.join(REPO, "tools", "gen_libm_tables.py"), str(hdr)], check=True)
    exe = tmp_path / "check_libm_ref"
    subprocess.run(["g++", "-O2", "-std=c++17", "-fno-builtin", "-ffp-contract=off", f"-I{tmp_path}",
                    f"-I{os.path.join(REPO, 'reinforcement-learning-101_amd', 'csrc')}",
                    os.path.join(REPO, "tools", "check_libm_ref.cpp"), "-o", str(exe), "-lm"], check=True)
    out = subprocess.run([str(exe), "1"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:]
    assert "0 / 4000015 differ" in out.stdout and "sin: 0 /" in out.stdout, out.stdout
