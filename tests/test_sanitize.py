"""The product's host-only code under AddressSanitizer + UndefinedBehaviorSanitizer
("run [the CPU path's] unit tests under -fsanitize=address,undefined").

tests/cpp/sanitize_test.cc links the per-object C-ABI (hyperdex_amd/csrc/hdx_cpu.cpp)
and the device set's cut rule (hdx_cuts.h) with the oracle as the checker, every
value in a heap buffer of exactly its length; built here with g++ (no GPU)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc/g++")
def test_cpu_path_and_cuts_under_asan_ubsan(tmp_path):
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
    inc = ["-I" + os.path.join(ROOT, "hyperdex_amd", "csrc"), "-I" + os.path.join(ROOT, "oracle"),
           "-I" + os.path.join(ROOT, "include")]
    oracle_o = str(tmp_path / "hdx_oracle.o")
    subprocess.run(["gcc", "-std=c11", *san, *inc, "-c", os.path.join(ROOT, "oracle", "hdx_oracle.c"), "-o", oracle_o],
                   check=True, timeout=300)
    exe = str(tmp_path / "sanitize_test")
    subprocess.run(["g++", "-std=c++17", *san, *inc, os.path.join(ROOT, "tests", "cpp", "sanitize_test.cc"),
                    os.path.join(ROOT, "hyperdex_amd", "csrc", "hdx_cpu.cpp"), oracle_o, "-o", exe, "-lpthread", "-lm"],
                   check=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "sanitize_test ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
