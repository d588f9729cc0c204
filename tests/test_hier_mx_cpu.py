"""Cross-node OCP MX compression of the hierarchical communicator (parallel/hierarchical.py
_cross_all_reduce_mx) on CPU: 3 gloo ranks act as 3 nodes; every rank must end with the node-order sum of
the MX-rounded shards, bitwise equal on all ranks."""
import os
import socket

import pytest
import torch


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, wire, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist

        from allreduce_over_mpi_amd.ops.quant import mx_round
        from allreduce_over_mpi_amd.parallel.hierarchical import HierarchicalCommunicator

        dist.init_process_group("gloo", rank=rank, world_size=world)
        hc = object.__new__(HierarchicalCommunicator)  # only the cross-node step: no intra-node communicator
        hc._torch, hc._dist, hc.nodes = torch, dist, world
        hc.cross_group, hc.cross_pg, hc.cross_on_host = dist.group.WORLD, None, True
        xs = [torch.randn(1000, generator=torch.Generator().manual_seed(r)) * 10 ** r for r in range(world)]
        y = hc._cross_all_reduce_mx(xs[rank].clone(), wire)
        want = mx_round(xs[0], wire)
        for x in xs[1:]:
            want = want + mx_round(x, wire)
        outs = [torch.empty_like(y) for _ in range(world)]
        dist.all_gather(outs, y)
        same = all(torch.equal(o, outs[0]) for o in outs)
        dist.destroy_process_group()
        q.put((rank, int((y != want).sum()), same, None))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, None, None, traceback.format_exc()))


@pytest.mark.parametrize("wire", ["e4m3", "e5m2"])
def test_cross_node_mx_sum(wire):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 3, port, wire, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(3)]
    for p in ps:
        p.join(30)
    for rank, mism, same, tb in res:
        assert tb is None, tb
        assert mism == 0 and same, (rank, mism, same)


def test_mx_cross_step_only_for_narrow_floats_and_few_nodes(monkeypatch):
    """float64 (and integer) shards take the exact cross-node path; the MX all-gather grows
    linearly with the node count, so beyond FLEXAR_HIER_MX_MAX_NODES (4) nodes the exact ring runs."""
    from allreduce_over_mpi_amd.parallel.hierarchical import HierarchicalCommunicator

    hc = object.__new__(HierarchicalCommunicator)
    hc._torch = torch
    for nodes, dt, want in [(2, torch.float32, True), (4, torch.bfloat16, True), (3, torch.float16, True),
                            (2, torch.float64, False), (2, torch.int32, False), (5, torch.float32, False)]:
        hc.nodes = nodes
        assert hc._mx_applies(dt) is want, (nodes, dt)
    monkeypatch.setenv("FLEXAR_HIER_MX_MAX_NODES", "8")
    hc.nodes = 5
    assert hc._mx_applies(torch.float32) is True
