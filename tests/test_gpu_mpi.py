"""MPI_Allreduce_FT on DEVICE buffers (real MI355X): the MPI layer routes hipMalloc'd buffers
to the flexar GPU engine (handles exchanged with MPI_Allgather, IPC between the ranks' processes),
or — when ranks do not share a node (forced with FLEXAR_MPI_P2P=1) — stages through host memory
and the point-to-point engine. Driven through the reference-compatible benchmark CLI with --check.
Also the RCCL comparator of the benchmark (ncclAllReduce) at one rank."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tools(cuda):
    from allreduce_over_mpi_amd import _build

    if not _build.mpi_available():
        pytest.skip("MPI not available")
    return _build.build_tools(["flexar_bench"])


def _mpirun(n, args, env=None):
    from allreduce_over_mpi_amd import _build

    e = dict(os.environ)
    e.update({"FLEXAR_MAX_GRID": "16", "FLEXAR_TIMEOUT_MS": "20000"})
    e.update(env or {})
    return subprocess.run([os.path.join(_build.MPI_HOME, "bin", "mpirun"), "-np", str(n)] + args,
                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300, env=e)


@pytest.mark.parametrize("algo", ["flat", "ring", "ll", "oneshot", "flat+zc"])
def test_mpi_device_buffers_ipc(tools, algo):
    r = _mpirun(2, [tools["flexar_bench"], "--mem", "device", "--size", "100003", "--repeat", "5", "--check",
                    "--algo", algo])
    assert r.returncode == 0 and "check n=100003: ok" in r.stdout, r.stdout[-3000:]


def test_mpi_zero_copy_sweep_reregisters(tools):
    """FLEXAR_ALGO=flat+zc through MPI_Allreduce_FT: every sweep size is a fresh hipMalloc (often at a
    freed buffer's address), so the MPI layer must (re-)register collectively and drop stale mappings."""
    r = _mpirun(2, [tools["flexar_bench"], "--mem", "device", "--sweep", "4K:4M", "--repeat", "3", "--check",
                    "--algo", "flat+zc"])
    assert r.returncode == 0 and r.stdout.count(": ok") >= 11, r.stdout[-3000:]
    r = _mpirun(2, [tools["flexar_bench"], "--mem", "device", "--dtype", "bfloat16", "--size", "65539", "--check",
                    "--algo", "flat+zc"])
    assert r.returncode == 0 and "check n=65539: ok" in r.stdout, r.stdout[-3000:]


def test_mpi_zero_copy_by_default(tools):
    """with no FLEXAR_ALGO, MPI_Allreduce_FT on device buffers of at least 1 MiB registers them
    collectively (mpi_mod.hpp zc_prepare) and the cost model's flat choice runs zero copy ("+zc+push"); below
    1 MiB, or with FLEXAR_MPI_ZC=0, or with a named spec, it runs staging. Results exact every time."""
    r = _mpirun(2, [tools["flexar_bench"], "--mem", "device", "--size", "4M", "--repeat", "5", "--check"])
    assert r.returncode == 0 and "check n=4194304: ok" in r.stdout, r.stdout[-3000:]
    sched = [ln for ln in r.stdout.splitlines() if ln.startswith("schedule n=4194304")]
    assert sched and "+zc" in sched[-1], r.stdout[-3000:]
    r = _mpirun(2, [tools["flexar_bench"], "--mem", "device", "--size", "4099", "--repeat", "3", "--check"])
    assert r.returncode == 0 and "check n=4099: ok" in r.stdout and "+zc" not in r.stdout, r.stdout[-3000:]
    for env, args in (({"FLEXAR_MPI_ZC": "0"}, []), ({}, ["--algo", "flat+pull"])):
        r = _mpirun(2, [tools["flexar_bench"], "--mem", "device", "--size", "4M", "--repeat", "3", "--check"] + args,
                    env=env)
        sched = [ln for ln in r.stdout.splitlines() if ln.startswith("schedule n=4194304")]
        assert r.returncode == 0 and sched and "+zc" not in sched[-1], (env, args, r.stdout[-3000:])


def test_mpi_zero_copy_default_fresh_buffers(tools):
    """The default registration with a fresh hipMalloc per sweep size (often a freed buffer's address): the
    per-call agreement catches stale registrations and re-registers; every size exact; bf16 too."""
    r = _mpirun(2, [tools["flexar_bench"], "--mem", "device", "--sweep", "256K:16M", "--repeat", "3", "--check"])
    assert r.returncode == 0 and r.stdout.count(": ok") >= 7, r.stdout[-3000:]
    # --sweep takes bytes: 2 MiB .. 16 MiB run zero copy (1 MiB and below: the selector picks LL)
    assert sum("+zc" in ln for ln in r.stdout.splitlines() if ln.startswith("schedule")) >= 4, r.stdout[-3000:]
    r = _mpirun(2, [tools["flexar_bench"], "--mem", "device", "--dtype", "bfloat16", "--size", "2M", "--check"])
    assert r.returncode == 0 and "check n=2097152: ok" in r.stdout, r.stdout[-3000:]


def test_mpi_zero_copy_refused_registration(tools):
    """A buffer whose registration is refused (its allocation above FLEXAR_REG_MAX_ALLOC, here 4 MiB) runs staging,
    exactly, and is not retried; buffers that fit keep running zero copy."""
    r = _mpirun(2, [tools["flexar_bench"], "--mem", "device", "--sweep", "2M:16M", "--repeat", "3", "--check"],
                env={"FLEXAR_REG_MAX_ALLOC": str(4 << 20)})
    assert r.returncode == 0 and r.stdout.count(": ok") >= 4, r.stdout[-3000:]
    sched = {int(ln.split("=")[1].split(":")[0]): ln.split(": ")[1] for ln in r.stdout.splitlines()
             if ln.startswith("schedule n=")}
    assert "+zc" in sched[(2 << 20) // 4] or "+zc" in sched[(4 << 20) // 4], sched
    assert "+zc" not in sched[(8 << 20) // 4] and "+zc" not in sched[(16 << 20) // 4], sched


def test_mpi_device_buffers_host_staging(tools):
    """Ranks on 'different nodes' (virtual nodes of 1 rank): whole buffer staged through host p2p."""
    r = _mpirun(2, [tools["flexar_bench"], "--mem", "device", "--size", "65537", "--repeat", "3", "--check"],
                env={"FLEXAR_NODE_SIZE": "1", "FLEXAR_MPI_FLAT_STAGING": "1", "FLEXAR_MPI_P2P": "1"})
    assert r.returncode == 0 and "check n=65537: ok" in r.stdout, r.stdout[-3000:]


@pytest.mark.parametrize("size", ["1", "7", "100003"])
def test_mpi_device_hierarchical(tools, size):
    """4 ranks as 2 virtual nodes x 2: intra-node reduce-scatter (flexar/IPC) -> inter-node host p2p
    allreduce of the shard -> intra-node all-gather; plus the < L-element tail."""
    r = _mpirun(4, [tools["flexar_bench"], "--mem", "device", "--size", size, "--repeat", "3", "--check"],
                env={"FLEXAR_NODE_SIZE": "2", "FLEXAR_MPI_P2P": "1"})
    assert r.returncode == 0 and f"check n={size}: ok" in r.stdout, r.stdout[-3000:]


def test_bench_bf16_and_rccl_comparator(tools):
    r = _mpirun(2, [tools["flexar_bench"], "--mem", "device", "--dtype", "bfloat16", "--size", "4099", "--check"])
    assert r.returncode == 0 and "check n=4099: ok" in r.stdout, r.stdout[-3000:]
    r = _mpirun(1, [tools["flexar_bench"], "--mem", "device", "--comm-type", "rccl", "--size", "1M", "--repeat", "5",
                    "--check"])
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-3000:]
