"""Standalone C++ tests of the platform core (native/tests/core_tests.cpp):
plain, ThreadSanitizer and ASan+UBSan builds.

The stress case runs 8 scheduler threads (schedule / extender filter+bind /
partition auto-provision / release) against topology refresh, the
housekeeping tick with zero-hysteresis partition reclaim, and metric
scrapes; it checks that no GPU or slice ever has two owners.  It caught the
idle-check -> mode-switch window that the partition-switch fence closes.
"""
from __future__ import annotations

import os
import subprocess

import pytest

from kgwe import _build


@pytest.mark.parametrize("flavour,iters", [("plain", 2000), ("tsan", 400), ("asan", 400)])
def test_core_native_suite(flavour, iters):
    try:
        exe = _build.build_native_tests(flavour, jobs=4)
    except RuntimeError as e:  # toolchain without the sanitizer runtime
        if flavour != "plain" and "sanitize" in str(e):
            pytest.skip(f"{flavour} runtime unavailable: {str(e)[-200:]}")
        raise
    env = dict(os.environ)
    env["TSAN_OPTIONS"] = "halt_on_error=1 second_deadlock_stack=1"
    env["ASAN_OPTIONS"] = "detect_leaks=1:halt_on_error=1:verify_asan_link_order=0"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    r = subprocess.run([str(exe), str(iters)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "all passed" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr
