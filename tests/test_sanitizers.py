"""ASan + UBSan build of the host-side C/C++ (liblbm_host's lbm_host.cpp and the oracle's
lbm_oracle.c) from source, driven through every entry point by tests/sanitize/host_sanitize.cpp:
out-of-bounds reads in the geometry builders, readers and writers fail the test.  (GPU code is
not sanitised: GPU AddressSanitizer is not available on the MI355X pool.)"""
import os
import shutil
import subprocess

import pytest

from conftest import GOLDEN, PKG, REPO


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_under_asan_ubsan(tmp_path):
    exe = tmp_path / "host_sanitize"
    flags = ["-O1", "-g", "-static-libasan", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
             "-ffp-contract=off"]
    oracle_o = tmp_path / "lbm_oracle.o"
    subprocess.run(["gcc", "-std=c11", "-c", *flags, os.path.join(REPO, "oracle", "lbm_oracle.c"), "-o",
                    str(oracle_o)], check=True, timeout=300)
    subprocess.run(["g++", "-std=c++17", *flags, os.path.join(REPO, "tests", "sanitize", "host_sanitize.cpp"),
                    os.path.join(PKG, "csrc", "lbm_host.cpp"), str(oracle_o), "-o", str(exe), "-lm"],
                   check=True, timeout=300)
    bif = os.path.join(GOLDEN, "bifurcation")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), os.path.join(bif, "geo.txt"), os.path.join(bif, "bc.txt"), str(tmp_path)],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "sanitize ok" in r.stdout, r.stderr[-4000:]
