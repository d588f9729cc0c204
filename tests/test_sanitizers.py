"""ASan + UBSan build of the host code (planner, host executor, simulator, host reduce) — CPU only."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_host_code_asan_ubsan(tmp_path):
    exe = tmp_path / "asan_simulate"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-I" + os.path.join(REPO, "csrc", "include"), os.path.join(REPO, "tests", "cpp", "asan_simulate.cpp"),
           os.path.join(REPO, "csrc", "src", "capi_host.cpp"), "-o", str(exe), "-lpthread"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=900, env=env)
    assert r.returncode == 0 and "0 failures" in r.stdout, r.stdout[-4000:]


def test_program_validator_host(tmp_path):
    """validate_program accepts every planner program and rejects each kind of corruption (host C++)."""
    exe = tmp_path / "validate_program"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-I" + os.path.join(REPO, "csrc", "include"), os.path.join(REPO, "tests", "cpp", "validate_program.cpp"),
           "-o", str(exe)]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    r = subprocess.run([str(exe)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0 and " 0 failures" in r.stdout, r.stdout[-4000:]
