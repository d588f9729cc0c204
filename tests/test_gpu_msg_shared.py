"""The RCCL message transport with real messages on a 1-GPU box.

RCCL refuses two ranks on one GPU of one host ("Duplicate GPU detected"), so test_gpu_msg.py can only run
the one-rank route and test_gpu_multidevice.py needs 2+ GPUs. RCCL decides "same host" from a hash of
NCCL_HOSTID when that is set: giving every process its own NCCL_HOSTID makes the ranks look like separate
hosts, and RCCL carries their messages over its socket network transport on the loopback interface. The
GPU, the executor segments, the arena and the grouped ncclSend / ncclRecv of run_msg (comm.hip) are then the
production ones; only RCCL's own wire differs from xGMI. This is the device twin of the host P2P engine
(csrc/include/flexar/mpi_mod.hpp, the reference's Isend/Irecv exchange at mpi_mod.hpp:662-765 of
/root/reference/allreduce_over_mpi) with more than one rank.

Covered: the connect-time self-test of the rccl family, every schedule with "+rccl" (flat, ring, RHD,
FlexTree 2x2) on fp32 / bf16 / uneven tails / SUM and AVG, three consecutive calls with changing inputs,
reduce-scatter / all-gather over the transport, and the automatic fallback when no peer can be mapped over
IPC (FLEXAR_FAULT_NO_IPC: every call, named spec or not, runs over RCCL).
"""
import os
import queue
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


def _worker(rank, world, port, specs, q, transport, no_ipc):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000",
                          # one "host" per rank: RCCL's socket transport over loopback, no duplicate-GPU refusal
                          NCCL_HOSTID=f"flexar-test-rank{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
        if no_ipc:
            os.environ["FLEXAR_FAULT_NO_IPC"] = "1"
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import Communicator

        comm = Communicator(workspace_bytes=64 << 20, transport=transport)
        dev = torch.device("cuda", 0)
        res = {"topology": comm.topology(), "selftest_failed": list(comm.selftest_failed)}
        for spec in specs:
            for dtype in (torch.float32, torch.bfloat16):
                for size in (5, 4099, 300007):
                    xs = [torch.randint(-64, 64, (size,), generator=torch.Generator().manual_seed(31 * r + size))
                          .to(dtype) for r in range(world)]
                    ref = torch.stack([x.double() for x in xs]).sum(0)
                    for op in ("sum", "avg"):
                        worst = 0.0
                        for s in (1.0, 0.5, 0.25):  # exact in every dtype: integers times powers of two
                            x = (xs[rank].double() * s).to(dtype).to(dev)
                            y = comm.all_reduce(x, op=op, algo=spec)
                            torch.cuda.synchronize()
                            want = ref * s / (world if op == "avg" else 1)
                            err = ((y.double().cpu() - want).abs().max() / (want.abs().max() + 1e-12)).item()
                            worst = max(worst, err)
                        res[(spec, str(dtype), size, op)] = worst
        # reduce-scatter / all-gather of m elements per rank over the same transport
        m = 10007
        xs = [torch.randint(-64, 64, (world * m,), generator=torch.Generator().manual_seed(r)).float()
              for r in range(world)]
        rs_algo = "flat+rccl" if transport == "rccl" else None
        rs = torch.empty(m, device=dev)
        ag = torch.empty(world * m, device=dev)
        comm.reduce_scatter(xs[rank].to(dev), rs, algo=rs_algo)
        comm.all_gather(xs[rank][:m].to(dev), ag, algo=rs_algo)
        torch.cuda.synchronize()
        want_rs = torch.stack(xs).sum(0)[rank * m:(rank + 1) * m]
        want_ag = torch.cat([x[:m] for x in xs])
        res["reduce_scatter"] = (rs.cpu() - want_rs).abs().max().item()
        res["all_gather"] = (ag.cpu() - want_ag).abs().max().item()
        comm.check()
        res["stats"] = {k: v for k, v in comm.stats().items() if isinstance(v, (int, float, str))}
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, None, traceback.format_exc()))


def _run(world, specs, transport, no_ipc):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, specs, q, transport, no_ipc)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=100)
            assert err is None, f"rank {rank} failed:\n{err}"
            out[rank] = res
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    except queue.Empty:
        pytest.fail(f"message transport with {world} ranks did not finish within 100 s")
    finally:
        for p in procs:  # a hung rank must not outlive the test on the GPU
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_rccl_message_transport_shared_gpu(cuda, world):
    specs = ["flat+rccl", "ring+rccl", "oneshot+rccl"]
    specs += ["rhd+rccl", "tree:2,2+rccl"] if world == 4 else []
    out = _run(world, specs, "rccl", False)
    for rank, res in out.items():
        topo, failed = res.pop("topology"), res.pop("selftest_failed")
        assert topo["rccl"] is True and topo["ipc"] is True, topo
        assert "rccl" in topo["selftested"].split(",") and failed == [], (topo, failed)
        res.pop("stats")
        for key, err in res.items():
            assert err == 0.0, (rank, key, err)  # integer-valued inputs: every dtype is exact


def test_rccl_fallback_without_ipc_shared_gpu(cuda):
    """No peer mapping on any rank (FLEXAR_FAULT_NO_IPC): the communicator comes up on the message
    transport alone and runs the FlexTree / ring / RHD / flat schedules over it, named or chosen."""
    world = 4
    specs = [None, "flat", "ring", "rhd", "tree:2,2", "oneshot"]
    out = _run(world, specs, "auto", True)
    for rank, res in out.items():
        topo, failed = res.pop("topology"), res.pop("selftest_failed")
        assert topo["ipc"] is False and topo["rccl"] is True, topo
        # the peer-memory families cannot run without mappings (reported as failed, calls avoid them); the
        # message transport is the one that ran and passed
        assert topo["selftested"] == "rccl" and "rccl" not in failed, (topo, failed)
        res.pop("stats")
        for key, err in res.items():
            assert err == 0.0, (rank, key, err)
