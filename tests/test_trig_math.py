"""CPU: the kernel's angle math (reinforcement-learning-101_amd/csrc/trig.h),
compiled for the host with g++, against glibc and the reference's loops.

* dd::trig::sincos vs glibc sin/cos (what numpy calls for the reference):
  never more than 1 ulp apart on the angles step() produces (about 13 % of
  results 1 ulp off: the reduction keeps no tail word, trig.h).
* dd::trig::div_exact vs IEEE division: bit-identical for the obs divisors.
* dd::trig::normalize_angle vs the reference's while-loops (physics.py:26-39):
  bit-identical, including multi-turn angles.
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRIG = os.path.join(REPO, "reinforcement-learning-101_amd", "csrc", "trig.h")

DRIVER = r"""
#include "TRIG_H"
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
static int64_t ulps(double a, double b) {
  int64_t ia, ib; std::memcpy(&ia, &a, 8); std::memcpy(&ib, &b, 8);
  if (ia < 0) ia = INT64_MIN - ia;
  if (ib < 0) ib = INT64_MIN - ib;
  return ia > ib ? ia - ib : ib - ia;
}
static double loop_wrap(double a) {  // physics.normalize_angle
  while (a > 180) a -= 360;
  while (a < -180) a += 360;
  return a;
}
int main() {
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> deg(-180.0, 180.0), wide(-2e5, 2e5), pos(-1e3, 1e3);
  const double d2r = 3.14159265358979323846 / 180.0;
  long n = 2000000, mism = 0; int64_t worst = 0;
  for (long i = 0; i < n; ++i) {
    double a = deg(g);
    if (i % 3 == 0) a = (float)a;
    if (i % 7 == 0) a = std::nearbyint(a * 8) / 8;
    double x = a * d2r, s, c;
    dd::trig::sincos(x, &s, &c);
    int64_t ds = ulps(s, std::sin(x)), dc = ulps(c, std::cos(x));
    mism += (ds != 0) + (dc != 0);
    if (ds > worst) worst = ds;
    if (dc > worst) worst = dc;
  }
  std::printf("sincos %ld %ld %lld\n", 2 * n, mism, (long long)worst);
  const double ds[] = {800, 600, 10, 180, 1000, 5000};
  long dmis = 0, dn = 0;
  for (double d : ds) {
    const double inv = 1.0 / d;
    for (long i = 0; i < 400000; ++i) {
      double x = (i & 1) ? pos(g) : wide(g);
      if (i % 5 == 0) x = (float)x;
      if (i % 11 == 0) x = std::ldexp(pos(g), -(int)(i % 900));
      dmis += dd::trig::div_exact(x, d, inv) != x / d;
      ++dn;
    }
  }
  std::printf("div %ld %ld\n", dn, dmis);
  long wmis = 0, wn = 0;
  for (long i = 0; i < 1000000; ++i) {
    double a = (i % 4 == 0) ? wide(g) : (i % 4 == 1) ? deg(g) * 2.0 : (i % 4 == 2) ? std::nearbyint(wide(g)) : pos(g);
    if (i % 9 == 0) a = 180.0 * (double)((long)(i % 41) - 20);  // exact multiples of 180
    if (i % 13 == 0) a = std::nextafter(180.0 * (double)((long)(i % 41) - 20), (i & 1) ? 1e9 : -1e9);
    wmis += dd::trig::normalize_angle(a) != loop_wrap(a);
    ++wn;
  }
  std::printf("wrap %ld %ld\n", wn, wmis);
}
"""


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    d = tmp_path_factory.mktemp("trig")
    src = d / "driver.cpp"
    src.write_text(DRIVER.replace("TRIG_H", TRIG))
    exe = d / "driver"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    return {line.split()[0]: [int(v) for v in line.split()[1:]] for line in out.strip().splitlines()}


def test_sincos_within_one_ulp_of_glibc(results):
    total, mism, worst = results["sincos"]
    assert worst <= 1
    assert mism / total < 0.16, mism / total


def test_div_exact_is_ieee_division(results):
    total, mism = results["div"]
    assert total > 0 and mism == 0


def test_normalize_angle_equals_reference_loops(results):
    total, mism = results["wrap"]
    assert total > 0 and mism == 0
