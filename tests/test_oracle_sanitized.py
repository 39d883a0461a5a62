"""CPU: the oracle's whole path under AddressSanitizer + UBSan (oracle/sanitize_main.c,
built by `make -C oracle san`): RNG primitives, the three bag regimes, subspaces, split
finding with and without Spark's split-finding sample, variance and gini fits, both
aggregations.  Any memory error, leak or undefined behaviour fails the run.  (The
product's host code runs under host ASan on the GPU box: tests/test_gpu_c_abi.py.)"""
import os
import subprocess

from conftest import ROOT


def test_oracle_clean_under_asan_ubsan():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san"])
    exe = os.path.join(ROOT, "oracle", "_san", "oracle_san")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    assert "oracle sanitizer run ok" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr
