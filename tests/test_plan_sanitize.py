"""The launch planner (host C++, csrc/bm_plan.cpp) under AddressSanitizer
and UBSan: tools/plan_fuzz.cpp plans thousands of random (msg, range) cases,
checks tiling / layout invariants and replays segments against a direct
SHA-256 of "msg nonce".  Host code only: GPU sanitizers are not available
on this pool."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_planner_fuzz_under_asan_ubsan(tmp_path):
    exe = tmp_path / "plan_fuzz"
    csrc = os.path.join(ROOT, "distributed_bitcoin_minter_amd", "csrc")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=all", "-I", csrc, "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tools", "plan_fuzz.cpp"), os.path.join(csrc, "bm_plan.cpp"),
                           "-o", str(exe)])
    r = subprocess.run([str(exe), "2000"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok"), r.stdout
