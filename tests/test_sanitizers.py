"""The C-ABI's host code and the C oracle under AddressSanitizer + UBSan (CPU only).

tests/asan/Makefile compiles every csrc/*.hip with the sanitizers on the host side
(-Xarch_host) and oracle/cs_oracle.c, and links tests/asan/host_abi_check.cpp, which
drives what runs on the host without a GPU: cs_prefix_attention_plan over 3,000 random
decode / scoring shapes (entries in range, split slots written once, exact-size plan
buffers), the split and workspace planners at extreme sizes, the argument checks of every
entry point, and known answers of the oracle.  Any invalid access, leak or undefined
behaviour fails the run.
"""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ASAN = os.path.join(HERE, "asan")


@pytest.fixture(scope="module")
def binary():
    r = subprocess.run(["make", "-C", ASAN, "-j8"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return os.path.join(ASAN, "host_abi_check")


def _run(binary, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    return subprocess.run([binary, *args], capture_output=True, text=True, timeout=300, env=env)


def test_host_code_is_clean_under_asan_and_ubsan(binary):
    r = _run(binary, "3000")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "host ABI checks passed" in r.stdout


def test_the_build_is_sanitized(binary):
    """An intentional heap overflow must be caught (the checks above ran instrumented)."""
    r = _run(binary, "overflow")
    assert r.returncode != 0 and "AddressSanitizer" in r.stderr, r.stderr[-2000:]
