"""The kernels' division-free pixel-centre / ray uv (soc_device.hpp div_rn) is the IEEE quotient: tools/check_div_rn.c
checks it exhaustively (every a = x + 0.5 with x < n and a = x with x <= n, n <= 16384; ~268 M quotients, <1 s)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_div_rn_exhaustive(tmp_path):
    exe = str(tmp_path / "check_div_rn")
    subprocess.run(["gcc", "-O2", "-mfma", os.path.join(ROOT, "tools", "check_div_rn.c"), "-o", exe, "-lm"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    assert "centre mismatches 0, integer mismatches 0" in r.stdout
