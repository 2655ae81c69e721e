"""The full detector's host-side keypoint order (removeDuplicatedSorted's
KeypointGreater, slam-indoor-code_amd/csrc/kp_order.h): its radix form
(kp_order) against std::sort with the comparator, on the CPU (ties in x and in
every field, signed zeros, negative x).  The detector's GPU parity tests check
the same order end to end against oracle/siftdet.c."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_kp_order_matches_std_sort(tmp_path):
    exe = str(tmp_path / "kp_order_test")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tests", "cpp", "kp_order_test.cpp")],
                   check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout + r.stderr
