"""The geometric moving average's pow (graphite_amd/csrc/glibc_pow.h) against
this image's glibc pow, bit for bit, on the host (CPU test).

MovingGeometricMean::compute (moving_average.h:119-135) chains pow() results,
so the engine carries glibc 2.35's algorithm (__pow_fma, e_pow.c) with the same
FMA contraction and tables.  tests/cpp/test_pow.cc compares it with ::pow over
~4.5 M operands: the walk's own (integer cycles ^ 1/w, mean ^ w, products),
random finite doubles, results near overflow / the subnormal range, and special
operands (0, inf, nan, negative x), plus the x86-64 double -> uint64 conversion
the reference's (T) _geometric_mean performs.  The same header is compiled into
libgnoc.so with -ffp-contract=off; IEEE operations give the same bits there
(the GPU test test_basic_moving_average checks the engine end to end)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pow_matches_glibc(tmp_path):
    exe = str(tmp_path / "test_pow")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-mfma", "-I" + os.path.join(ROOT, "graphite_amd", "csrc"),
                    "-o", exe, os.path.join(ROOT, "tests", "cpp", "test_pow.cc"), "-lm"], check=True)
    r = subprocess.run([exe, "1000000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "pow: 0 of" in r.stdout and "cast: 0 differ" in r.stdout, r.stdout
