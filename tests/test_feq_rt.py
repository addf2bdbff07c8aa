"""feq_rt (run-time q, the NEE path of k_step) against the reference's per-q expression
trees feq<q> / feq_bc<q> (ldc.cu:330-348, Poiseulle.cu:543-561, bifurcation.cu:587-624;
boundary tmp terms ldc.cu:402-454), bit for bit on the host (same IEEE fp32 operations,
no contraction) -- tools/feq_rt_check.cpp."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not found")
def test_feq_rt_bitwise(tmp_path):
    exe = tmp_path / "feq_rt_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                    os.path.join(REPO, "tools", "feq_rt_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "100000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches 0" in out.stdout
