"""Production path across processes: one process per rank, workspaces mapped
through HIP IPC, bootstrap through torch.distributed (gloo). On the 1-GPU box
every rank uses device 0 (IPC between processes on one device exercises the
same handle exchange, mapping and system-scope flag protocol as xGMI peers).
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, specs, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000")
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import Communicator

        comm = Communicator(workspace_bytes=64 << 20)
        dev = torch.device("cuda", 0)
        results = {}
        for spec in specs:
            for size in (7, 4096, 300001):
                xs = [torch.randn(size, generator=torch.Generator().manual_seed(100 * r + size)) for r in range(world)]
                ref = torch.stack(xs).double().sum(0)
                x = xs[rank].to(dev)
                for _ in range(3):
                    y = comm.all_reduce(x.clone(), algo=spec)
                torch.cuda.synchronize()
                err = (y.double().cpu() - ref).abs().max().item()
                results[(spec, size)] = err
        comm.check()
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, results, None))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 4])
def test_ipc_allreduce_processes(cuda, world):
    import torch.multiprocessing as mp

    specs = ["flat", "flat+push", "ring", "ring:2", "oneshot"] + (["rhd", "tree:2,2+push"] if world == 4 else [])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, specs, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, res, err = q.get(timeout=300)
        assert err is None, f"rank {rank} failed:\n{err}"
        out[rank] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res in out.items():
        for key, err in res.items():
            assert err < 1e-4, (rank, key, err)
