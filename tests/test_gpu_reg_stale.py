"""A stale registration on one rank only (comm_reg.hip / reg_lookup).

Both ranks register their buffer X. Rank 1 then frees X and allocates a fresh X2 of the same size (the
allocator hands back the same addresses once the cache is emptied), while rank 0 keeps X. Both register Y
= the same sub-range of their current buffer: rank 1 drops its stale registration of X (its allocation is
gone), rank 0 keeps X's (still valid, larger, containing Y). A zero-copy call on Y must bind through the
NEWEST registration on every rank - Y's - or rank 0 would read rank 1's old X through a stale mapping.
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000")
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import Communicator

        comm = Communicator(workspace_bytes=64 << 20)
        n = 8 << 20  # 32 MiB: its own segment of the caching allocator
        x = torch.zeros(n, device=dev)
        comm.register(x)
        old_ptr = x.data_ptr()
        if rank == 1:
            del x
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            x = torch.zeros(n, device=dev)  # a new allocation (usually at the same address)
        lo, m = 1 << 20, 1 << 18
        y = x[lo:lo + 2 * m]
        comm.register(y)
        out = {"reused": x.data_ptr() == old_ptr, "regs": comm._lib.flexar_reg_count(comm._h)}
        errs = []
        for call in range(3):
            src = y[:m]
            dst = y[m:2 * m]
            src.copy_(torch.arange(m, device=dev, dtype=torch.float32) * (rank + 1) + call)
            comm.all_reduce(src, out=dst, algo="flat+zc+push")
            torch.cuda.synchronize()
            want = torch.arange(m, device=dev, dtype=torch.float32) * 3 + 2 * call
            errs.append(float((dst - want).abs().max().item()))
        out["err"] = max(errs)
        comm.check()
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, None, traceback.format_exc()))


def test_stale_registration_on_one_rank(cuda):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, out, err = q.get(timeout=180)
        assert err is None, f"rank {rank}:\n{err}"
        res[rank] = out
    for p in procs:
        p.join(timeout=60)
    for rank, out in res.items():
        assert out["err"] == 0.0, (rank, out)
    # rank 0 still holds X's registration next to Y's; rank 1 dropped its stale one when the address was reused
    assert res[0]["regs"] == 2
    if res[1]["reused"]:
        assert res[1]["regs"] == 1, res
