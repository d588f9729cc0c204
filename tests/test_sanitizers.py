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


@pytest.mark.slow
def test_host_executor_tsan(tmp_path):
    """ThreadSanitizer over the same simulator driver: the host executor runs every workgroup of every rank as
    its own thread and orders them only through the programs' SIGNAL / WAIT flags and the staging parity, so a
    schedule whose flags do not order a reader after its writer (a missing wait, a slot reused one call too
    early, a channel sharing another's slots) is reported as a data race on the staging or output bytes."""
    exe = tmp_path / "tsan_simulate"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread",
           "-I" + os.path.join(REPO, "csrc", "include"), os.path.join(REPO, "tests", "cpp", "asan_simulate.cpp"),
           os.path.join(REPO, "csrc", "src", "capi_host.cpp"), "-o", str(exe), "-lpthread"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    r = subprocess.run([str(exe)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=1200, env=env)
    assert r.returncode == 0 and "0 failures" in r.stdout, r.stdout[-4000:]
    assert "ThreadSanitizer" not in r.stdout, r.stdout[-4000:]


def test_host_executor_tsan_negative_control(tmp_path):
    """The TSAN verdict above is only worth something if a missing WAIT is caught: rhd:3+pull at N = 4 runs
    clean as planned and is reported as a data race once rank 0's channel 1 stops waiting for its peers."""
    exe = tmp_path / "tsan_negative"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-I" + os.path.join(REPO, "csrc", "include"),
           os.path.join(REPO, "tests", "cpp", "tsan_negative.cpp"), "-o", str(exe), "-lpthread"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    r = subprocess.run([str(exe)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ok rc=0" in r.stdout, r.stdout[-4000:]
    r = subprocess.run([str(exe), "drop"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300,
                       env=env)
    assert r.returncode == 66 and "ThreadSanitizer: data race" in r.stdout, r.stdout[-4000:]
    assert "host_reduce_span" in r.stdout or "memcpy" in r.stdout or "host_xfer" in r.stdout, r.stdout[-4000:]


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
