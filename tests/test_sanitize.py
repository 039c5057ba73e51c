"""CPU: the host engine (csrc/engine.cpp and the host side of every .hip launcher) under
AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 "race detection / sanitizers").

`make -C multimodal-drl-rmc_amd sanitize` builds host-only objects (no device code) with
-fsanitize=address,undefined and links tests/sanitize/plan_check.cpp, which plans ~270 engine
configurations without a GPU: every network family, algorithm, dtype, batch and data-parallel
split, their arena layouts, learn-step launch lists for every flag set, DP bucket cuts, acting /
sampler scratch sizes and the refusal paths.  Any sanitizer report aborts the program.
(It found two reads of the engine's config after `delete e` on create's error paths.)"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "multimodal-drl-rmc_amd")


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and shutil.which("hipcc") is None,
                    reason="needs hipcc (host-only compile)")
def test_host_engine_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", PKG, "-j8", "sanitize"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(PKG, "build", "plan_check")], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert ", 0 failures" in r.stdout, out[-2000:]
