"""The collective-teardown agreement (csrc/src/host_barrier.hpp) on the CPU: N processes meet on one
shared-memory page for several phases, in any arrival order; a rank that never arrives makes its peers
return FLEXAR_ERR_TIMEOUT naming it instead of hanging; the page's name is removed.

The reference never frees its scratch (allreduce_over_mpi/mpi_mod.hpp:931-950), so it has no teardown to
agree on; flexar_comm_destroy runs these barriers between drain, unmap and free (docs/DESIGN.md §21)."""
import multiprocessing as mp
import os
import time
import uuid

import pytest


def _run(name, rank, world, phases, timeout_ms, delay_ms, q):
    from allreduce_over_mpi_amd import _native as nv

    lib = nv.lib()
    t0 = time.monotonic()
    rc = lib.flexar_host_barrier_run(name.encode(), rank, world, phases, timeout_ms, delay_ms)
    q.put((rank, rc, nv.last_error() if rc else "", time.monotonic() - t0))


def _spawn(world, phases, timeout_ms, delays, absent=()):
    name = f"/flexar.test.{os.getpid()}.{uuid.uuid4().hex[:12]}"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_run, args=(name, r, world, phases, timeout_ms, delays[r], q))
             for r in range(world) if r not in absent]
    for p in procs:
        p.start()
    out = {}
    for _ in procs:
        r, rc, err, dt = q.get(timeout=60)
        out[r] = (rc, err, dt)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    return name, out


@pytest.mark.parametrize("world", [2, 4, 8])
def test_barrier_phases_any_arrival_order(world):
    # staggered arrivals (rank r is r * 15 ms late at every phase): everyone passes every phase
    name, out = _spawn(world, 4, 20000, [15 * r for r in range(world)])
    assert sorted(out) == list(range(world))
    for r, (rc, err, _) in out.items():
        assert rc == 0, (r, err)
    assert not os.path.exists("/dev/shm" + name), "rank 0 removes the name after the first phase"


def test_barrier_names_the_absent_rank():
    # rank 2 of 3 never arrives: ranks 0 and 1 time out within the limit and name it
    name, out = _spawn(3, 2, 800, [0, 0, 0], absent=(2,))
    for r in (0, 1):
        rc, err, dt = out[r]
        assert rc == 4, (r, rc, err)  # FLEXAR_ERR_TIMEOUT
        assert "rank 2 did not arrive" in err, err
        assert 0.7 < dt < 10.0, dt
    assert not os.path.exists("/dev/shm" + name)


def _page(name, rank, world, token, bdir, q):
    from allreduce_over_mpi_amd import _native as nv
    from allreduce_over_mpi_amd.parallel.comm import file_exchange
    import ctypes

    lib = nv.lib()
    ex = file_exchange(bdir, rank, world, timeout_s=60)
    h = lib.flexar_host_page_open(name.encode(), rank, world, token)
    ex(b"")  # the bootstrap barrier after connect (every rank has marked)
    t0 = time.monotonic()
    missing = ctypes.c_int(-1)
    shared = lib.flexar_host_page_shared(h, token, ctypes.byref(missing))
    dt = time.monotonic() - t0
    ex(b"")
    lib.flexar_host_page_close(h)
    q.put((rank, shared, missing.value, dt))


@pytest.mark.parametrize("private", [False, True])
def test_page_shared_check_is_immediate(private, tmp_path):
    """at connect each rank writes a mark into the page; after one bootstrap barrier every
    rank checks every mark. Ranks that joined different pages (one container per rank: a private /dev/shm,
    simulated by per-rank names) learn it at once, not by an agreement timing out at teardown."""
    world = 3
    base = f"/flexar.test.{os.getpid()}.{uuid.uuid4().hex[:12]}"
    token = 0x1234_5678_9ABC_DEF0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_page, args=(base + (f".r{r}" if private else ""), r, world, token,
                                             str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in procs:
        r, shared, missing, dt = q.get(timeout=90)
        out[r] = (shared, missing, dt)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r, (shared, missing, dt) in out.items():
        assert shared == (0 if private else 1), (r, out)
        assert dt < 0.5, (r, dt)
        if private:
            assert missing != r and 0 <= missing < world, (r, missing)
