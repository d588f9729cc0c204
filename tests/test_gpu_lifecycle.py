"""Communicator lifecycle on the device: separate processes on one GPU (IPC,
gloo bootstrap), like tests/test_gpu_calibration.py.

* close() is collective inside the library (flexar_comm_destroy: drain -> agree -> unmap -> agree -> free),
  so ranks may close and build communicators back to back with NO caller barrier, arriving at different
  times, and every result stays exact;
* a rank whose peer never reaches the teardown returns after FLEXAR_TIMEOUT_MS with a named error, and
  keeps its exported workspace allocated instead of freeing memory a peer may still map;
* a HIP error in one rank's self-test launch (FLEXAR_TEST_SELFTEST_HIP, test-only: an invalid block size)
  fails that family on EVERY rank with the error named, the protocol state is resynchronised, the
  downgrade chain goes on, and later calls are exact;
* a failure every rank agrees on at connect (every device protocol failed the self-test) closes the
  communicator collectively and builds it once more in the same process (transport "auto").

Reference contrast: allreduce_over_mpi/mpi_mod.hpp:931-950 (scratch that is never freed while in use).
"""
import glob
import os
import socket
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _exact(comm, rank, world, n, algo=None, salt=0):
    dev = torch.device("cuda", 0)
    x = (torch.arange(n, device=dev, dtype=torch.int32) % 977 + rank + salt).float()
    y = comm.all_reduce(x.clone(), algo=algo)
    want = (torch.arange(n, device=dev, dtype=torch.int32) % 977).float() * world + world * (world - 1) / 2 \
        + world * salt
    return float((y - want).abs().max().item())


def _worker(rank, world, port, mode, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000", FLEXAR_CALIB="0")
        if mode == "hiperr":
            os.environ["FLEXAR_TEST_SELFTEST_HIP"] = f"{world - 1}:1"  # last rank: fence launches fail
        if mode == "retry":
            os.environ["FLEXAR_TEST_SELFTEST_HIP"] = "0:15:1"  # rank 0, every IPC family, first communicator
        if mode == "absent":
            os.environ["FLEXAR_TIMEOUT_MS"] = "2000"
        if mode == "private":  # every rank joins a page of its own (a private /dev/shm per container)
            os.environ["FLEXAR_TEST_PAGE_PRIVATE"] = "1"
            os.environ["FLEXAR_TIMEOUT_MS"] = "8000"
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import Communicator

        out = {}
        if mode == "rebuild":
            errs = []
            dev = torch.device("cuda", 0)
            x = torch.empty(1 << 20, device=dev)
            y = torch.empty(1 << 20, device=dev)
            for cyc in range(3):
                comm = Communicator(workspace_bytes=64 << 20)  # no barrier before: close() agreed already
                comm.register_many([x, y])
                for algo in (None, "flat+pull", "ring", "ll", "flat+zc+push"):
                    n = 4096 if algo == "ll" else (1 << 20)
                    x[:n].copy_((torch.arange(n, device=dev, dtype=torch.int32) % 977 + rank + cyc).float())
                    comm.all_reduce(x[:n], out=y[:n], algo=algo)
                    want = (torch.arange(n, device=dev, dtype=torch.int32) % 977).float() * world \
                        + world * (world - 1) / 2 + world * cyc
                    errs.append(float((y[:n] - want).abs().max().item()))
                comm.check()
                time.sleep(0.05 * rank)  # ranks reach the teardown at different times
                comm.close()  # and no barrier after
            out["err"] = max(errs)
        elif mode == "absent":
            comm = Communicator(workspace_bytes=64 << 20)
            out["err"] = _exact(comm, rank, world, 1 << 18)
            comm.check()
            dist.barrier()
            if rank == world - 1:
                comm.close(collective=False)  # never reaches the agreement
            else:
                from allreduce_over_mpi_amd import _native as nv

                t0 = time.monotonic()
                comm.close()
                out["close_s"] = time.monotonic() - t0
                out["parked"] = int(nv.lib().flexar_parked_bytes())
            dist.barrier()
        elif mode == "private":
            comm = Communicator(workspace_bytes=64 << 20)
            topo = comm.topology()
            out["page"] = (topo["host_page"], topo["host_page_shared"], comm.host_page_note)
            out["err"] = _exact(comm, rank, world, 1 << 18)
            comm.check()
            t0 = time.monotonic()
            comm.close()  # no page: the two teardown agreements run over the bootstrap exchange
            out["close_s"] = time.monotonic() - t0
            for _ in range(2):  # and again: nothing is ever parked
                c2 = Communicator(workspace_bytes=64 << 20)
                out["err"] = max(out["err"], _exact(c2, rank, world, 1 << 16))
                c2.close()
            from allreduce_over_mpi_amd import _native as nv

            out["parked"] = int(nv.lib().flexar_parked_bytes())
        elif mode in ("hiperr", "retry"):
            comm = Communicator(workspace_bytes=64 << 20)
            out["failed"] = list(comm.selftest_failed)
            out["notes"] = {int(k): v for k, v in comm.selftest_notes.items()}
            out["retried"] = comm.retried
            out["disabled"] = comm.topology()["disabled"]
            out["err"] = max(_exact(comm, rank, world, n, algo, salt=k)
                             for k, (n, algo) in enumerate([(1000, None), (1 << 18, None), (1 << 20, "flat+pull"),
                                                            (1 << 20, "ring"), (4096, "ll")]))
            comm.check()
            comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, None, traceback.format_exc()))


def _run(world, mode):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=240)
            assert err is None, f"rank {rank} failed:\n{err}"
            out[rank] = res
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return out, [p.pid for p in procs]


@pytest.mark.parametrize("world", [2, 4])
def test_close_and_rebuild_without_caller_barrier(cuda, world):
    out, pids = _run(world, "rebuild")
    for r in range(world):
        assert out[r]["err"] == 0.0, (r, out[r])
    # every teardown page was removed (names carry rank 0's pid)
    assert not glob.glob(f"/dev/shm/flexar.{pids[0]}.*")


def test_close_with_an_absent_peer_times_out_named(cuda):
    out, _ = _run(2, "absent")
    assert out[0]["err"] == 0.0 and out[1]["err"] == 0.0
    assert 1.5 < out[0]["close_s"] < 15.0, out[0]
    assert out[0]["parked"] >= 64 << 20, out[0]  # the timed-out close parks (and says so: a warning)


def test_private_host_page_is_detected_at_connect(cuda):
    """ranks that do not share /dev/shm are told at connect (not by a teardown timeout):
    the page is dropped on every rank, calls stay exact and close() returns without waiting out
    FLEXAR_TIMEOUT_MS (8 s here)."""
    out, _ = _run(2, "private")
    for r in range(2):
        o = out[r]
        assert o["page"][0] is False and o["page"][1] is False, (r, o)
        assert o["err"] == 0.0, (r, o)
        assert o["close_s"] < 4.0, (r, o)
        assert o["parked"] == 0, (r, o)  # the workspace is freed, not parked for the process's life
    assert "host page not shared" in (out[0]["page"][2] or ""), out[0]


@pytest.mark.parametrize("world", [2, 4])
def test_selftest_hip_error_downgrades_on_every_rank(cuda, world):
    out, _ = _run(world, "hiperr")
    bad = world - 1
    for r in range(world):
        o = out[r]
        assert o["failed"] == ["fence"], (r, o)
        assert "fence" in o["disabled"], (r, o)
        note = " ".join(o["notes"].get(bad, []))
        assert "selftest_fill launch" in note and "flat+pull call 0" in note, (r, o["notes"])
        assert o["err"] == 0.0, (r, o)
        assert o["retried"] is None


def test_agreed_connect_failure_is_retried_once(cuda):
    out, _ = _run(2, "retry")
    for r in range(2):
        o = out[r]
        assert o["retried"] and "no device protocol passed" in o["retried"], (r, o)
        assert o["failed"] == [] and o["disabled"] == "", (r, o)
        assert o["err"] == 0.0, (r, o)
