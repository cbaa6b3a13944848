"""Host-side native code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU, no GPU).

Builds tests/native/planner_check.cpp — the planner arithmetic libevam_pp.so shares with its kernels
(csrc/evam_geom.h: ROI clipping and geometry, OpenCV coefficient entries, staged footprints, LDS
staging bounds, algorithmic bytes, ROI launch order) — together with the C oracle, both with
``-fsanitize=address,undefined -fno-sanitize-recover=all``, and runs it. The checks compare the
planner with the oracle's geometry over random and extreme (int32-overflowing) rects, check every
staging bound it computes against brute force, and drive the oracle on exactly-sized frame
allocations so an out-of-bounds read in either fails the test.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1",
       "-ffp-contract=off"]


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc/g++")
def test_planner_and_oracle_under_asan_ubsan(tmp_path):
    obj = tmp_path / "oracle.o"
    exe = tmp_path / "planner_check"
    subprocess.run(["gcc", *SAN, "-std=c11", "-c", os.path.join(ROOT, "oracle", "evam_oracle.c"), "-o", str(obj)],
                   check=True)
    subprocess.run(["g++", *SAN, "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "planner_check.cpp"), str(obj), "-o", str(exe), "-lm"],
                   check=True)
    # verify_asan_link_order=0: the environment may preload its own library ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "all checks passed" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_descriptor_rings_under_asan_ubsan(tmp_path):
    """The pinned ROI-record ring and the descriptor upload ring (csrc/evam_rings.h, the code evam_pp_run
    runs) against a simulated device timeline: no host write, copy or free of a slot while an enqueued
    kernel may still read it, over slot reuse across the run-of-4 fences, capacity growth, stream switches
    and failed calls; the negative controls (no event waits; failed calls left undrained) must
    report violations."""
    exe = tmp_path / "ring_check"
    subprocess.run(["g++", *SAN, "-std=c++17", os.path.join(ROOT, "tests", "native", "ring_check.cpp"), "-o",
                    str(exe)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "all checks passed" in r.stdout and "rings: 8000 calls" in r.stdout and " 0 violations" in r.stdout
