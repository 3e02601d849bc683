"""The C ABI from a compiled C caller (tests/c_abi/abi_driver.c): include/casim.h and
libcasim.so only, no Python binding in between — what a cgo shim links against
(INTEGRATION.md).  CPU: it compiles and links; GPU: it runs every check."""
import os
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c_abi")
BIN = os.path.join(HERE, "bin", "abi_driver")


def test_driver_builds_against_header_and_library():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    assert os.path.exists(BIN)
    syms = subprocess.run(["nm", "-D", "--undefined-only", BIN], check=True, capture_output=True, text=True).stdout
    assert "ca_estimate_batch" in syms and "ca_find_nodes_to_remove" in syms and "ca_mirror_remove_node" in syms


@pytest.mark.gpu
def test_driver_runs():
    if not os.path.exists(BIN):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_driver ok" in r.stdout
    assert "estimate node_count 125 n_scheduled 1000" in r.stdout


def test_intern_driver_against_fixtures():
    """The interning through casim.h alone, from C, against tests/golden/intern_calls.txt
    (the calls and the ids / encodings tests/golden/intern_fixtures.json pins).  Host-only:
    runs on the CPU."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    calls = os.path.join(os.path.dirname(HERE), "golden", "intern_calls.txt")
    r = subprocess.run([os.path.join(HERE, "bin", "intern_driver"), calls], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "intern_driver ok" in r.stdout
