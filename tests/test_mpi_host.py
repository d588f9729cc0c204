"""MPI_Allreduce_FT on host buffers (the reference's own domain) — CPU only.

Runs the C++ harness tests/cpp/test_mpi_allreduce.cpp under MPICH
(`mpirun -np N`, oversubscribed on this host): every algorithm, several dtypes
and ops, in/out of place, against the vendor MPI_Allreduce. Both host engines:
the shared-memory window engine and the point-to-point message engine
(FLEXAR_MPI_P2P=1, the multi-node path).
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def tools(nv):
    from allreduce_over_mpi_amd import _build

    if not _build.mpi_available():
        pytest.skip("MPI not available")
    return _build.build_tools(["test_mpi_allreduce", "flexar_bench", "flexar_plan"])


def _mpirun():
    from allreduce_over_mpi_amd import _build

    p = os.path.join(_build.MPI_HOME, "bin", "mpirun")
    return p if os.path.exists(p) else shutil.which("mpirun")


def _run(args, env=None, timeout=300):
    e = dict(os.environ)
    e.update(env or {})
    e.pop("FLEXAR_ALGO", None) if not (env and "FLEXAR_ALGO" in env) else None
    return subprocess.run(args, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=timeout, env=e)


@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_mpi_shared_memory_engine(tools, n):
    r = _run([_mpirun(), "-np", str(n), tools["test_mpi_allreduce"]] + (["--quick"] if n == 8 else []))
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout[-3000:]


@pytest.mark.parametrize("n", [2, 5, 6])
def test_mpi_p2p_engine(tools, n):
    r = _run([_mpirun(), "-np", str(n), tools["test_mpi_allreduce"], "--quick"], env={"FLEXAR_MPI_P2P": "1"})
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout[-3000:]


def test_benchmark_cli_reference_compatible(tools):
    """benchmark.cpp CLI: --size --repeat --comm-type --tag --to-file, CHECK and DONE lines (host buffers)."""
    r = _run([_mpirun(), "-np", "2", tools["flexar_bench"], "--mem", "host", "--size", "1024", "--repeat", "20",
              "--check", "--comm-type", "flextree"], env={"FT_TOPO": "1"})
    assert r.returncode == 0, r.stdout[-2000:]
    assert "DONE, average time:" in r.stdout and "CHECK 0:" in r.stdout and "check n=1024: ok" in r.stdout
    r = _run([_mpirun(), "-np", "2", tools["flexar_bench"], "--mem", "host", "--size", "35", "--comm-type", "mpi"])
    assert r.returncode == 0 and "DONE" in r.stdout
    r = _run([tools["flexar_bench"], "--version"])
    assert "flexar standalone benchmark" in r.stdout
    r = _run([tools["flexar_bench"], "--bogus"])
    assert r.returncode != 0


def test_plan_tool(tools):
    r = _run([tools["flexar_plan"], "model", "8", "100"])
    assert "should be (reference model): 8" in r.stdout, r.stdout
    r = _run([tools["flexar_plan"], "dump", "tree:2,4", "8", "5", "64"])
    assert "SIGNAL" in r.stdout and "rank 5" in r.stdout
    r = _run([tools["flexar_plan"], "choose", "7"])
    assert "2*4-1" in r.stdout and "2*3+1" in r.stdout
    r = _run([tools["flexar_plan"], "sweep", "20"])
    assert r.stdout.splitlines()[0] == "N,structures,microseconds" and len(r.stdout.splitlines()) == 21


def test_plan_tool_link_table(tools):
    """flexar_plan links: per phase, the bytes rank 0 moves with each peer. rhd:7 at N = 8 drives all 7 links in every
    phase with equal bytes; single-channel rhd drives one."""
    def table(spec):
        r = _run([tools["flexar_plan"], "links", spec, "8", str(64 << 20)])
        assert r.returncode == 0, r.stdout
        rows = [ln.split() for ln in r.stdout.splitlines()[2:]]
        return [[float(v) for v in row[2:]] for row in rows]
    seven = [row for row in table("rhd:7+pull") if any(row)]  # (the pull form has one phase of local work only)
    assert len(seven) == 6
    for row in seven:
        assert all(v > 0 for v in row) and max(row) - min(row) <= 0.01 * max(row), row
    one = [row for row in table("rhd+pull") if any(row)]
    assert len(one) == 6 and all(sum(v > 0 for v in row) == 1 for row in one), one
