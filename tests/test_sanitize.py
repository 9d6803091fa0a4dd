"""The C ABI's host code under AddressSanitizer and UndefinedBehaviorSanitizer.

`make sanitize` builds tests/native/sanitize_driver.cpp against the library's host objects
compiled with -Xarch_host -fsanitize=address,undefined (device code untouched) and the C oracle as
the checker.  Host-only checks run here; with a GPU the driver also checks process_chunk,
process_chunks, the basic strategy and run_tokenizer against the oracle, with 8 threads sharing a
handle.  Any sanitizer report aborts the driver (non-zero exit).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "build", "san", "blt_sanitize_driver")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


_BUILT = []


def _driver():
    """`make sanitize` once per session, every session: make rebuilds the driver whenever a source
    it is built from changed (round 4 only built it when absent, and a stale driver reported false
    device failures after the library's host code changed)."""
    if not _BUILT:
        r = subprocess.run(["make", "-C", ROOT, "-j8", "sanitize"], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        _BUILT.append(True)
    return DRIVER


def test_sanitize_driver_rebuilt_when_stale():
    """The driver is up to date with the library's host sources after _driver() (make -q: nothing
    left to rebuild)."""
    _driver()
    r = subprocess.run(["make", "-C", ROOT, "-q", "sanitize"], capture_output=True)
    assert r.returncode == 0


def test_host_checks_under_asan_ubsan():
    r = subprocess.run([_driver(), "--cpu"], capture_output=True, text=True, env=ENV, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host checks: 0 failure(s)" in r.stdout


@pytest.mark.gpu
def test_device_checks_under_asan_ubsan():
    # Under ASan the HIP runtime's start-up fails in some processes (its address-space reservations
    # and ASan's shadow mappings collide, by layout): the driver's probe then gets BLT_E_NODEV, says
    # "no HIP device" and runs the host checks only.  A fresh process gets a fresh layout: up to five
    # tries for that one start-up error.  Any other probe failure is a driver failure (the probe
    # reports it), and so is a runtime that never starts on a box whose GPU the plain suite sees: the
    # device checks never turn into a skip.
    import torch
    for _ in range(5):
        r = subprocess.run([_driver()], capture_output=True, text=True, env=ENV, timeout=300)
        if "no HIP device" not in r.stdout:
            break
    else:
        assert not torch.cuda.is_available(), "HIP runtime did not start under ASan in five processes: " + r.stdout
        pytest.skip("no GPU")
    # the first failures name the cause (later ones follow from it): the head of the report too
    assert r.returncode == 0, r.stdout[-1500:] + r.stderr[:2500] + "\n...\n" + r.stderr[-1500:]
    assert "host and device checks: 0 failure(s)" in r.stdout, r.stdout
