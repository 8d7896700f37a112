"""The compile-time GF(2^16) arithmetic of the GF(2^16) encoder (gf16_constexpr.hpp) is
the oracle's field: products, the twiddle = index structure of the skew table, the
GF(2^8) subfield and (a, b) coordinates, the v_perm / bit-matrix tables, and the lane
decomposition of the twiddles the plane layers 2-4 rely on (rs_gf16x.hip layer_p). Host only."""
import os
import subprocess


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gf16_constexpr_matches_oracle(oracle, tmp_path):
    exe = tmp_path / "gf16_check"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-o", str(exe),
                           os.path.join(ROOT, "tests", "gf16_constexpr_check.cpp"),
                           "-L", os.path.join(ROOT, "oracle"), "-loracle",
                           "-Wl,-rpath," + os.path.join(ROOT, "oracle")])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr
