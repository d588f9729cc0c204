"""One process per GPU (the production topology): every rank on its own device, workspaces mapped
across devices through HIP IPC over xGMI, bootstrap through torch.distributed (gloo).

A 1-GPU box skips this module (tests/test_gpu_ipc.py covers the same protocol with every process on
device 0). On a multi-GPU node it checks every algorithm family against a float64 host reference on
fp32/bf16, uneven tail sizes, SUM and the fused AVG post-scale, with inputs that change every call
(x, x/2, x/4 on alternating staging parities) so a stale staging line cannot go unnoticed.
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ngpu() -> int:
    try:
        return torch.cuda.device_count()
    except Exception:
        return 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, specs, q, transport="rccl", no_ipc=False):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_TIMEOUT_MS="20000")
        if no_ipc:
            os.environ["FLEXAR_FAULT_NO_IPC"] = "1"  # every peer mapping fails: the RCCL fallback carries all
        import torch.distributed as dist

        torch.cuda.set_device(rank)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import Communicator

        comm = Communicator(workspace_bytes=128 << 20, transport=transport)
        dev = torch.device("cuda", rank)
        results = {}
        for spec in specs:
            for dtype in (torch.float32, torch.bfloat16):
                for size in (5, 4096, 1000003):
                    xs = [torch.randn(size, generator=torch.Generator().manual_seed(100 * r + size)).to(dtype)
                          for r in range(world)]
                    ref = torch.stack([x.double() for x in xs]).sum(0)
                    for op in ("sum", "avg"):
                        worst = 0.0
                        for s in (1.0, 0.5, 0.25):
                            x = (xs[rank].double() * s).to(dtype).to(dev)
                            y = comm.all_reduce(x, op=op, algo=spec)
                            torch.cuda.synchronize()
                            want = ref * s / (world if op == "avg" else 1)
                            err = ((y.double().cpu() - want).abs().max() / (want.abs().max() + 1e-12)).item()
                            worst = max(worst, err)
                        results[(spec, str(dtype), size, op)] = worst
        if not no_ipc:  # zero copy across devices: peers read / write registered buffers over xGMI
            for dtype in (torch.float32, torch.bfloat16):
                arena = torch.empty(1000003, device=dev, dtype=dtype)
                out = torch.empty_like(arena)
                comm.register_many([arena, out])
                for spec in ("flat+zc", "flat+zc+push", "flat+zc+push+wt", "flat+zc+put", "flat+zc+put+nts"):
                    for size in (5, 4096, 1000003):
                        xs = [torch.randn(size, generator=torch.Generator().manual_seed(7 * r + size)).to(dtype)
                              for r in range(world)]
                        ref = torch.stack([x.double() for x in xs]).sum(0)
                        for call in range(3):  # consecutive calls: the closing hand-off
                            arena[:size].copy_(xs[rank].to(dev))
                            comm.all_reduce(arena[:size], out=out[:size], algo=spec)
                        torch.cuda.synchronize()
                        err = ((out[:size].double().cpu() - ref).abs().max() / (ref.abs().max() + 1e-12)).item()
                        results[(spec, str(dtype), size, "sum")] = err
        comm.check()
        results["readiness"] = (comm.topology(), list(comm.selftest_failed))
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, results, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, None, traceback.format_exc()))


@pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (one process per device)")
def test_allreduce_one_process_per_gpu(cuda):
    import torch.multiprocessing as mp

    world = min(_ngpu(), 8)
    specs = ["flat", "flat+push", "flat+wt", "ring", "ring+wt", "oneshot", "ll", "dma", "flat+rccl", "ring+rccl",
             "flat+bidir", "flat+bidir+nts"]
    if world > 2:
        specs.append("ring:2")
    if world >= 4 and (world & (world - 1)) == 0:
        specs += ["rhd", "rhd+rccl"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, specs, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, res, err = q.get(timeout=600)
        assert err is None, f"rank {rank} failed:\n{err}"
        out[rank] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res in out.items():
        topo, failed = res.pop("readiness")
        # connect-time probe: every peer is another GPU reachable peer-to-peer; the self-test verified
        # every protocol family on the real links
        assert failed == [], (rank, failed, topo)
        assert topo["selftested"] == "fence,wt,ll,dma,rccl", topo
        for p in topo["peers"]:
            if p["rank"] != rank:
                assert p["link"] in ("xgmi", "pcie"), topo
                assert p["device"] == p["rank"], topo  # torch.cuda.set_device(rank) in _worker
        if all(p["link"] == "xgmi" and p["hops"] <= 1 for p in topo["peers"] if p["rank"] != rank):
            assert topo["links"] == world - 1, topo
        for key, err in res.items():
            tol = 1e-5 if "float32" in key[1] else 2e-2
            assert err < tol, (rank, key, err)


@pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (one RCCL rank per device)")
def test_rccl_fallback_when_ipc_is_unavailable(cuda):
    """Every peer mapping fails (FLEXAR_FAULT_NO_IPC): the communicator still comes up and every schedule
    (FlexTree, ring, RHD, flat) runs over the RCCL message transport with the same results."""
    import torch.multiprocessing as mp

    world = min(_ngpu(), 4)
    specs = ["flat", "ring", "oneshot"] + (["rhd", "tree:2,2"] if world == 4 else [])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, specs, q, "auto", True)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, res, err = q.get(timeout=600)
        assert err is None, f"rank {rank} failed:\n{err}"
        out[rank] = res
    for p in procs:
        p.join(timeout=60)
    for rank, res in out.items():
        topo, failed = res.pop("readiness")
        assert topo["ipc"] is False and topo["rccl"] is True, topo
        assert topo["selftested"] == "rccl" and "rccl" not in failed, (topo, failed)
        for key, err in res.items():
            tol = 1e-5 if "float32" in key[1] else 2e-2
            assert err < tol, (rank, key, err)
