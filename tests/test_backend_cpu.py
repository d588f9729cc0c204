"""The "flexar" c10d backend on CPU (gloo world of 2 processes): registration,
CPU-tensor allreduce/broadcast/allgather/barrier plumbing through the Python
ProcessGroup. (Device allreduce is covered by tests/test_gpu_backend.py.)"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist

        import allreduce_over_mpi_amd.parallel.backend as fb  # noqa: F401  registers "flexar"

        dist.init_process_group("flexar", rank=rank, world_size=world)
        assert dist.get_backend() == "flexar"
        x = torch.arange(10, dtype=torch.float32) * (rank + 1)
        dist.all_reduce(x)
        y = torch.tensor([rank + 1], dtype=torch.int64)
        dist.all_reduce(y, op=dist.ReduceOp.MAX)
        b = torch.tensor([float(rank)]) if rank == 0 else torch.tensor([-1.0])
        b[0] = 7.0 if rank == 0 else b[0]
        dist.broadcast(b, src=0)
        outs = [torch.zeros(2) for _ in range(world)]
        dist.all_gather(outs, torch.full((2,), float(rank)))
        r = torch.full((3,), float(rank + 1))
        dist.reduce(r, dst=1)  # CPU tensors: the fallback group's reduce (gloo leaves non-roots undefined)
        assert rank != 1 or r.tolist() == [3.0] * 3, r
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, x.tolist(), int(y.item()), float(b.item()), [o.tolist() for o in outs], None))
    except Exception:
        import traceback

        q.put((rank, None, None, None, None, traceback.format_exc()))


def test_flexar_backend_cpu_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in range(2)]
    for p in ps:
        p.join(60)
    for rank, x, y, b, outs, err in res:
        assert err is None, err
        assert x == [float(i * 3) for i in range(10)]
        assert y == 2 and b == 7.0
        assert outs == [[0.0, 0.0], [1.0, 1.0]]


def _fx_worker(d, rank, world, q):
    from allreduce_over_mpi_amd.parallel import file_exchange

    ex = file_exchange(d, rank, world)
    a = ex(f"hello{rank}".encode())
    b = ex(bytes([rank]) * (rank + 1))
    q.put((rank, a, b))


def test_file_exchange_rendezvous(tmp_path):
    """File-based bootstrap exchange: two all-gather rounds across 3 processes."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_fx_worker, args=(str(tmp_path), r, 3, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = dict((r, (a, b)) for r, a, b in (q.get(timeout=60) for _ in ps))
    for p in ps:
        p.join(30)
    for r in range(3):
        a, b = res[r]
        assert a == [b"hello0", b"hello1", b"hello2"]
        assert b == [b"\x00", b"\x01\x01", b"\x02\x02\x02"]


class _PageStub:
    """Stand-in for a device Communicator's host agreement (Communicator.host_agree_or: bitwise OR over the
    ranks of one 64-bit value), computed with a gloo BOR so the backend's bitmask logic runs on the CPU."""

    def __init__(self, has_page, pg):
        self.has_page, self.pg, self.calls = has_page, pg, 0

    def topology(self):
        return {"host_page": self.has_page}

    def host_agree_or(self, v):
        import torch.distributed as dist

        self.calls += 1
        t = torch.tensor([v], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.BOR, group=self.pg)
        return int(t.item())


def _agree_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist

        import allreduce_over_mpi_amd.parallel.backend as fb  # noqa: F401  registers "flexar"

        dist.init_process_group("flexar", rank=rank, world_size=world)
        pg = dist.group.WORLD
        side = dist.new_group(backend="gloo")
        out = {}
        for has_page in (True, False):
            pg._host_agree = None
            stub = _PageStub(has_page and True, side)
            # flag 1 is False on rank 0 only, flag 3 on rank 1 only, flag 5 everywhere; the others are True
            flags = [not ((i == 1 and rank == 0) or (i == 3 and rank == 1) or i == 5) for i in range(7)]
            got = pg._agree_all(flags, stub)
            out[has_page] = (got, stub.calls, pg._host_agree)
        dist.destroy_process_group()
        q.put((rank, out, None))
    except Exception:
        import traceback

        q.put((rank, None, traceback.format_exc()))


def test_backend_agreements_over_the_host_page_bitmask():
    """The zero-copy probe / sweep agreements (FlexarProcessGroup._agree_all): per flag, True only when it is
    True on every rank - through one host-page max over a bitmask of this rank's False flags when every rank
    has the page, else one gloo MIN."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_agree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in range(2)]
    for p in ps:
        p.join(60)
    for rank, out, err in res:
        assert err is None, err
        for has_page in (True, False):
            got, calls, mode = out[has_page]
            assert got == [True, False, True, False, True, False, True], (has_page, got)
            assert calls == (1 if has_page else 0) and mode is has_page


def _compress_worker(rank, world, port, settings, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_PG_COMPRESS=settings[rank])
        import torch.distributed as dist

        import allreduce_over_mpi_amd.parallel.backend as fb  # noqa: F401  registers "flexar"

        dist.init_process_group("flexar", rank=rank, world_size=world)
        pg = dist.group.WORLD
        try:
            picks = [pg._compress_algo(torch.zeros(1 << 20), "avg"),  # 4 MiB fp32: compressed
                     pg._compress_algo(torch.zeros(1 << 20, dtype=torch.bfloat16), "sum"),  # 2 MiB: too small
                     pg._compress_algo(torch.zeros(1 << 18, dtype=torch.int32), "sum"),
                     pg._compress_algo(torch.zeros(1 << 18), "max"),
                     pg._rs_algo(torch.zeros(1 << 21, dtype=torch.bfloat16), "avg"),  # reduce-scatter input
                     pg._rs_algo(torch.zeros(16), "sum")]
            err = None
        except RuntimeError as e:
            picks, err = None, str(e)
        dist.destroy_process_group()
        q.put((rank, picks, err, None))
    except Exception:
        import traceback

        q.put((rank, None, None, traceback.format_exc()))


@pytest.mark.parametrize("settings", [("mx_e4m3", "mx_e4m3"), ("mx_e4m3", "")])
def test_backend_compression_option_is_agreed(settings):
    """FLEXAR_PG_COMPRESS: float SUM / AVG allreduces of >= 4 MiB get the OCP MX wire; the setting is agreed
    on the first call and a mismatch fails on every rank (it would compile different schedules)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_compress_worker, args=(r, 2, port, settings, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in range(2)]
    for p in ps:
        p.join(60)
    for rank, picks, err, tb in res:
        assert tb is None, tb
        if settings[0] == settings[1]:
            assert err is None and picks == ["flat+pull+mxe4m3", None, None, None, "flat+pull+mxe4m3", None], \
                (rank, picks, err)
        else:
            assert picks is None and "differs across ranks" in err, (rank, picks, err)


class _PgStub:
    def __init__(self, algo, world):
        self.algo, self._world, self._rank = algo, world, 1
        self._compress_name, self._mx_carrier = "mx_e4m3", None


class _CommStub:
    def __init__(self, ipc):
        self.ipc = ipc

    def topology(self):
        return {"ipc": self.ipc}


@pytest.mark.parametrize("algo,world,ipc,want", [
    (None, 4, True, "flat+pull"),
    ("flat+push", 8, True, "flat+push"),
    ("flat+zc+push", 2, True, "flat+push"),  # the MX wire runs on staging: the zero-copy modifier is dropped
    ("tree:4", 4, True, "tree:4"),
    ("ring", 4, True, ""),              # the planner rejects a wire on a ring
    ("rhd", 8, True, ""),
    ("tree:2,4", 8, True, ""),
    ("oneshot", 4, True, ""),
    ("ll", 4, True, ""),
    (None, 9, True, ""),                # more than 8 ranks: one reduction of every contribution is impossible
    (None, 16, True, ""),
    ("flat+rccl", 4, True, ""),         # message transport
    (None, 4, False, ""),               # IPC unavailable: every call runs over RCCL
])
def test_backend_mx_wire_only_where_the_spec_carries_it(algo, world, ipc, want):
    """FLEXAR_PG_COMPRESS applies the MX suffix only to a flat schedule of 2..8 ranks over
    IPC; otherwise the call runs uncompressed instead of raising FlexarError inside the DDP / FSDP step."""
    from allreduce_over_mpi_amd.parallel.backend import FlexarProcessGroup

    pg = _PgStub(algo, world)
    got = FlexarProcessGroup._mx_carrier_spec(pg, _CommStub(ipc))
    assert got == want, (algo, world, ipc, got)
    assert FlexarProcessGroup._mx_carrier_spec(pg, None) == want  # decided once
