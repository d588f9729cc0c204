"""Fault attribution: a process that dies after recording flexar launches names them.

The native ring of breadcrumbs (csrc/src/crumbs.hpp) records every launch and phase; the fatal-signal and
std::terminate handlers print it with write(2) and chain to the previous handler. The reference's
counterpart is glog's InstallFailureSignalHandler (allreduce_over_mpi/benchmark.cpp:62). Here a child
process records a phase, attempts a reduction-kernel launch (no GPU on this host: the launch itself fails,
after its breadcrumb), records another phase and then dies by SIGABRT, SIGSEGV or std::terminate; its
stderr must carry the report with the launch and the last phase, and the process must still die by the
original signal (the handler chains). A stack overflow too: the handler runs on a
per-thread alternate signal stack, so the report still comes out of a thread whose own stack is exhausted.
"""
import os
import signal
import subprocess
import sys
import textwrap

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import ctypes, os, sys
    sys.path.insert(0, {repo!r})
    from allreduce_over_mpi_amd import _native as nv
    l = nv.lib()
    nv.crumb("bench", "phase: communicator ready", 1, 8)
    srcs = (ctypes.c_void_p * 2)(0x10000, 0x20000)
    l.flexar_reduce(ctypes.c_void_p(0x30000), srcs, 2, 4096, 0, 0, ctypes.c_float(1.0), None)
    nv.crumb("bench", "phase: last before the fault", 1, 8)
    how = {how!r}
    if how == "abort":
        os.abort()
    elif how == "segv":
        ctypes.string_at(0)
    elif how == "overflow":
        l.flexar_test_fatal(2)  # unbounded native recursion: the SIGSEGV arrives on an exhausted stack
    else:
        l.flexar_test_fatal(0)
""")


def _run(how, env_extra=None):
    env = dict(os.environ, FLEXAR_NO_BUILD="1", HIP_VISIBLE_DEVICES="")
    env.pop("FLEXAR_CRASH_REPORT", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "-c", CHILD.format(repo=REPO, how=how)], env=env, capture_output=True,
                          text=True, timeout=180)


@pytest.mark.parametrize("how,sig", [("abort", signal.SIGABRT), ("segv", signal.SIGSEGV), ("terminate", signal.SIGABRT),
                                     ("overflow", signal.SIGSEGV)])
def test_fatal_report_names_the_last_launch(how, sig):
    r = _run(how)
    assert r.returncode == -sig, (r.returncode, r.stderr[-2000:])
    err = r.stderr
    assert "[flexar crash report]" in err, err[-2000:]
    if how == "terminate":
        assert "std::terminate" in err
    report = err[err.index("[flexar crash report]"):]
    lines = [ln for ln in report.splitlines() if ln.startswith("[flexar crash report]   #")]
    launches = [ln for ln in lines if " launch " in ln]
    assert launches and "kernel=reduce" in launches[-1] and "float32/sum" in launches[-1] and "[flexar_reduce]" in launches[-1]
    assert "phase: last before the fault" in lines[-1]
    assert report.count("[flexar crash report] end") == 1  # one report, even when terminate -> abort chains


def test_report_can_be_disabled():
    r = _run("abort", {"FLEXAR_CRASH_REPORT": "0"})
    assert r.returncode == -signal.SIGABRT
    assert "[flexar crash report]" not in r.stderr
