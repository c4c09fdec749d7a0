"""include/hyperdex_amd/hash.h compiles as the daemon would use it (CPU), and
returns the reference's values through the GPU (gpu)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "dropin_test")


def build():
    subprocess.check_call([
        "g++", "-std=c++11", "-O2", "-Wall", "-Werror",
        "-I", os.path.join(ROOT, "tests", "cpp", "shim"), "-I", os.path.join(ROOT, "include"),
        os.path.join(ROOT, "tests", "cpp", "dropin_test.cc"), "-o", EXE,
        "-L", os.path.join(ROOT, "hyperdex_amd"), "-lhdxhash",
        "-Wl,-rpath," + os.path.join(ROOT, "hyperdex_amd")])


def test_dropin_header_compiles_and_links():
    build()
    assert os.path.exists(EXE)


@pytest.mark.gpu
def test_dropin_header_values_on_gpu():
    build()
    r = subprocess.run([EXE], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "dropin ok" in r.stdout
