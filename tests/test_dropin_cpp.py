"""include/hyperdex_amd/hash.h — the drop-in for common/hash.h — compiles
against the reference's own type headers, links, and returns the reference's
values on a host with no GPU (the per-object signatures run on the CPU inside
libhdxhash.so, hdx_cpu.cpp), at well under a microsecond per config-3b
object."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "dropin_test")
REF = "/root/reference"


def have_reference_headers():
    return all(os.path.exists(os.path.join(REF, p)) for p in
               ("common/schema.h", "common/attribute.h", "include/hyperdex.h", "namespace.h"))


def build(against_reference):
    if against_reference:
        # only libe's e/slice.h is a stand-in; schema / attribute / hyperdatatype
        # are the reference's own headers
        incs = ["-I", os.path.join(ROOT, "tests", "cpp", "shim_e"), "-I", REF, "-I", os.path.join(REF, "include")]
    else:
        incs = ["-I", os.path.join(ROOT, "tests", "cpp", "shim_e"), "-I", os.path.join(ROOT, "tests", "cpp", "shim_types")]
    subprocess.check_call(
        ["g++", "-std=c++11", "-O2", "-Wall", "-Werror"] + incs +
        ["-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "cpp", "dropin_test.cc"), "-o", EXE,
         "-L", os.path.join(ROOT, "hyperdex_amd"), "-lhdxhash", "-Wl,-rpath," + os.path.join(ROOT, "hyperdex_amd")])


@pytest.mark.skipif(not have_reference_headers(), reason="reference headers absent (GPU box)")
def test_dropin_against_reference_headers_on_cpu():
    build(True)
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "dropin ok" in r.stdout


def test_dropin_values_and_cost_on_cpu():
    build(have_reference_headers())
    r = subprocess.run([EXE, "bench", "2000000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "dropin ok" in r.stdout
    ns = float(re.search(r"ns_per_object ([0-9.]+)", r.stdout).group(1))
    # SURVEY §8b / VERDICT r1: well under 1 us per config-3b object on one core
    assert ns < 1000.0, r.stdout
