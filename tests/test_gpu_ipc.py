"""Production path across processes: one process per rank, workspaces mapped
through HIP IPC, bootstrap through torch.distributed (gloo). On the 1-GPU box
every rank uses device 0 (IPC between processes on one device exercises the
same handle exchange, mapping and system-scope flag protocol as xGMI peers).
"""
import os
import time
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

    specs = ["flat", "flat+push", "ring", "ring:2", "oneshot", "flat+wt", "flat+push+wt", "ring+wt", "dma", "flat+bidir",
             "flat+bidir+nts"]
    specs += ["rhd", "tree:2,2+push", "tree:2,2+wt"] if world == 4 else []
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


def _graph_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000")
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import Communicator

        comm = Communicator(workspace_bytes=32 << 20)
        dev = torch.device("cuda", 0)
        n = 200003
        x = torch.empty(n, device=dev)
        y = torch.empty(n, device=dev)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            x.fill_(float(rank + 1))
            comm.all_reduce(x, out=y)  # warm-up: compiles and uploads the plan before capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            comm.all_reduce(x, out=y)
            y.mul_(2.0)
            comm.all_reduce(y)  # in place, second call in the same graph
        errs = []
        for it in range(4):  # replays alternate staging parities through the device-side epochs
            x.fill_(float(rank + 1 + it))
            g.replay()
            torch.cuda.synchronize()
            want = 2.0 * world * sum(r + 1 + it for r in range(world))
            errs.append((y - want).abs().max().item())
        comm.check()
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, errs, None))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, None, traceback.format_exc()))


def test_ipc_allreduce_hip_graph_replay(cuda):
    """flexar_allreduce is graph-capturable: no host sync/alloc in the launch path, epochs live on device."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_graph_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    for rank, errs, tb in res:
        assert tb is None, tb
        assert max(errs) == 0.0, (rank, errs)


def _hier_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000")
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import HierarchicalCommunicator

        hc = HierarchicalCommunicator(node_size=2, workspace_bytes=32 << 20)  # 2 virtual nodes x 2 ranks
        dev = torch.device("cuda", 0)
        errs = []
        for size in (1, 3, 4097, 300001):
            xs = [torch.randn(size, generator=torch.Generator().manual_seed(10 * r + size)) for r in range(world)]
            st = torch.stack([x.double() for x in xs])
            for op, want in (("sum", st.sum(0)), ("avg", st.mean(0)), ("max", st.max(0).values)):
                y = hc.all_reduce(xs[rank].to(dev), op=op)
                torch.cuda.synchronize()
                errs.append((op, size, (y.double().cpu() - want).abs().max().item()))
        hc.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, errs, None))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, None, traceback.format_exc()))


def _hier_mx_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000")
        import torch.distributed as dist

        from allreduce_over_mpi_amd.ops.quant import mx_round

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import HierarchicalCommunicator

        hc = HierarchicalCommunicator(node_size=2, workspace_bytes=32 << 20)  # 2 virtual nodes x 2 ranks
        dev = torch.device("cuda", 0)
        errs = []
        for size, wire, op in ((4096, "mx_e4m3", "sum"), (300002, "mx_e4m3", "avg"), (65538, "mx_e5m2", "sum")):
            xs = [torch.randn(size, generator=torch.Generator().manual_seed(10 * r + size)) * (1 + r) for r in range(world)]
            m = size // 2
            want = torch.empty(size)
            for l in range(2):  # local rank l owns shard l: node sums (exact pairs), MX per node, node order
                sl = slice(l * m, (l + 1) * m)
                nodes = [xs[2 * k][sl] + xs[2 * k + 1][sl] for k in range(2)]
                want[sl] = mx_round(nodes[0], wire[3:]) + mx_round(nodes[1], wire[3:])
            if op == "avg":
                want.mul_(1.0 / world)
            y = hc.all_reduce(xs[rank].to(dev), op=op, compress=wire)
            torch.cuda.synchronize()
            exact = torch.stack([x.double() for x in xs]).sum(0) * (1.0 / world if op == "avg" else 1.0)
            rel = ((y.double().cpu() - exact).abs().max() / exact.abs().max()).item()
            errs.append((size, wire, int((y.cpu() != want).sum()), rel))
        hc.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, errs, None))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, None, traceback.format_exc()))


def test_hierarchical_allreduce_mx_cross_node(cuda):
    """compress="mx_e4m3"/"mx_e5m2": exact intra-node reduce-scatter, OCP MX fp8 shards all-gathered across the
    (virtual) nodes and summed in node order - bitwise the torch reference, the same on every rank."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hier_mx_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(4)]
    for p in procs:
        p.join(timeout=60)
    for rank, errs, tb in res:
        assert tb is None, tb
        for size, wire, mism, rel in errs:
            assert mism == 0, (rank, size, wire, mism)
            assert rel < (0.07 if wire == "mx_e4m3" else 0.13), (rank, size, wire, rel)


def test_hierarchical_allreduce_virtual_nodes(cuda):
    """Intra-node flexar RS/AG over IPC + cross-node allreduce of 1/L shards (2 virtual nodes x 2 ranks)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hier_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(4)]
    for p in procs:
        p.join(timeout=60)
    for rank, errs, tb in res:
        assert tb is None, tb
        for op, size, err in errs:
            assert err < 1e-4, (rank, op, size, err)


def _autotune_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000")
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import Communicator

        comm = Communicator(workspace_bytes=64 << 20)
        table = comm.autotune(sizes=[4096, 1 << 20, 8 << 20], iters=3)
        chosen = [comm.describe(b // 4, torch.float32).split(" ")[0] for b, _, _ in table]
        torch.manual_seed(5)  # same input on every rank
        x = torch.randn(300001, device="cuda")
        y = comm.all_reduce(x.clone())
        torch.cuda.synchronize()
        err = (y.double().cpu() - x.double().cpu() * world).abs().max().item()
        comm.set_tune_table("")  # back to the cost model
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, (table, chosen, err), None))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, None, traceback.format_exc()))


def test_autotune_installs_measured_table(cuda):
    """Communicator.autotune: validated, max-over-ranks timings; the installed winners drive auto calls."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_autotune_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    tables = []
    for rank, out, tb in res:
        assert tb is None, tb
        table, chosen, err = out
        assert len(table) == 3 and err < 1e-4, (table, err)
        for (b, spec, bw), ch in zip(table, chosen):  # describe() reports the installed choice ("flat" = tree:N)
            assert ch == spec.replace("flat", "tree:2"), (spec, ch)
        tables.append([s for _, s, _ in table])
    assert tables[0] == tables[1]  # every rank installed the same table


def _memo_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000", FLEXAR_PROFILE="1")
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import Communicator

        comm = Communicator(workspace_bytes=64 << 20)
        torch.manual_seed(9)  # same input on every rank
        x = torch.randn(1 << 18, device="cuda")
        ref = x.double().cpu() * world
        errs, seen = [], []

        def call(**kw):
            y = comm.all_reduce(x.clone(), **kw)
            torch.cuda.synchronize()
            errs.append((y.double().cpu() - ref).abs().max().item())
            seen.append(set(comm.stats()["profile"]))

        call()                           # auto: the cost model's choice
        call()                           # memo hit
        comm.set_algo("ring")
        call()                           # the default changed: must not reuse the memoised plan
        comm.set_tune_table(f"{world} 0 flat+push")
        comm.set_algo("auto")
        call()                           # auto again, now from the installed table
        call(algo="oneshot")             # same size, explicit algorithm
        call(algo="ring")
        comm.set_grid(4)
        call(algo="ring")                # grid override bumps the memo too
        comm.check()
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, (errs, [sorted(k) for k in seen]), None))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, None, traceback.format_exc()))


def test_plan_memo_follows_configuration_changes(cuda):
    """The per-communicator plan memo of flexar_allreduce_ex (a repeated call skips spec parsing and the
    program lookup) must be invalidated by set_algo / set_tune_table / set_grid: every call lands under
    the algorithm the current configuration selects (FLEXAR_PROFILE records per-algorithm device time)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_memo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    for rank, out, tb in res:
        assert tb is None, tb
        errs, seen = out
        assert max(errs) < 1e-4, errs
        # new algorithm names appear exactly where the configuration changed
        assert len(seen[0]) == 1 and seen[1] == seen[0], seen
        assert len(seen[2]) == 2 and any(k.startswith("ring") for k in seen[2]), seen
        assert len(seen[3]) == 3 and any("push" in k for k in seen[3]), seen
        assert len(seen[4]) == 3 + (0 if any(k.startswith("oneshot") for k in seen[3]) else 1), seen


def _captured_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000")
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import CapturedAllReduce, Communicator

        comm = Communicator(workspace_bytes=64 << 20)
        sizes = [64, 16384, 1 << 18, 300001]
        bufs = [torch.empty(n, device="cuda") for n in sizes]
        outs = [None, torch.empty(sizes[1], device="cuda"), None, None]
        comm.register(bufs[3])  # zero copy replays from a graph too (the peers' pointers are bound at capture)
        cap = CapturedAllReduce(comm, bufs, outs=outs, algo=[None, "oneshot", "dma", "flat+zc+push"])
        errs = []
        for it in range(5):
            xs = [[torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + 10 * r + k))
                   for r in range(world)] for k, n in enumerate(sizes)]
            for k, b in enumerate(bufs):
                b.copy_(xs[k][rank])
            cap.replay()
            torch.cuda.synchronize()
            for k, res in enumerate(cap.results):
                ref = torch.stack(xs[k]).double().sum(0)
                errs.append((res.double().cpu() - ref).abs().max().item())
        # eager calls after replays, dma included: the host never saw the replays' epochs
        x = torch.full((1 << 18,), float(rank + 1), device="cuda")
        for spec in ("dma", "flat", "ll"):
            y = comm.all_reduce(x.clone(), algo=spec)
            torch.cuda.synchronize()
            errs.append((y - world * (world + 1) / 2).abs().max().item())
        comm.check()
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, errs, None))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, None, traceback.format_exc()))


def test_captured_allreduce_replays(cuda):
    """CapturedAllReduce: LL / oneshot / dma-requested / zero-copy calls captured in one graph, replayed with
    new inputs; eager calls (dma included) stay correct afterwards."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_captured_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    for rank, errs, tb in res:
        assert tb is None, tb
        assert len(errs) == 23 and max(errs) < 1e-4, errs


def _stress_worker(rank, world, port, calls, q, fault=""):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000")
        if fault:
            os.environ["FLEXAR_FAULT_INJECT"] = fault
        import random

        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import Communicator

        comm = Communicator(workspace_bytes=32 << 20)
        specs = ["flat", "flat+push", "flat+wt", "flat+push+nts", "ring", "ring+wt", "oneshot", "ll", "dma",
                 "rhd", "tree:2,2+push", "flat+bidir", "rhd:3+pull", "tree:2,2:3+push"] if world == 4 else \
            ["flat", "flat+push+wt", "ring", "oneshot", "ll", "dma", "flat+bidir+wt"]
        if world == 8:  # link-balanced channelled trees (rhd:7 drives all 7 links in every stage)
            specs += ["rhd:7+pull", "tree:4,2:7+push"]
        specs += ["flat+zc", "flat+zc+push", "flat+zc+put"]
        # zero-copy calls run on registered arenas (the same offsets on every rank: the same call sequence)
        arena_in = torch.empty(world * 2_000_003 + 64, device="cuda")
        arena_out = torch.empty(world * 2_000_003 + 64, device="cuda")
        comm.register(arena_in)
        comm.register(arena_out)
        rnd = random.Random(1234)  # same call sequence on every rank
        side = torch.cuda.Stream()
        main = torch.cuda.current_stream()
        bad, pending = [], []
        for it in range(calls):
            spec = rnd.choice(specs)
            n = rnd.choice([1, 5, 4096, 65537, 300001, 2_000_003])
            in_place = rnd.random() < 0.5
            use_side = rnd.random() < 0.5
            # small integers in fp32: every summation order gives the exact same result
            gen = torch.Generator().manual_seed(it)
            allx = torch.randint(-8, 9, (world, max(n, world)), generator=gen).float()[:, :max(n, world)]
            x = allx[rank][:n].to("cuda")
            out = None if in_place else torch.empty_like(x)
            coll = rnd.choice(["allreduce"] * 4 + ["broadcast", "all_to_all", "reduce_scatter", "all_gather"])
            m = max(1, n // world)
            stream = side if use_side else main
            if coll == "allreduce":
                want = allx[:, :n].sum(0)
            elif coll == "broadcast":
                root = it % world
                want = allx[root][:n]
            elif coll == "all_to_all":
                x = allx[rank][:m * world].to("cuda")
                out = torch.empty_like(x)
                want = torch.cat([allx[r][rank * m:(rank + 1) * m] for r in range(world)])
            elif coll == "reduce_scatter":
                x = allx[rank][:m * world].to("cuda")
                out = torch.empty(m, device="cuda")
                want = allx[:, rank * m:(rank + 1) * m].sum(0)
            else:  # all_gather
                x = allx[rank][:m].to("cuda")
                out = torch.empty(m * world, device="cuda")
                want = allx[:, :m].reshape(-1)
            zc = "zc" in spec
            if zc:  # move the operands into the arenas once every earlier call on either stream is done
                main.wait_stream(side)
                off = it % 64  # a different (same-on-every-rank) offset each time
                ax = arena_in[off:off + x.numel()]
                ax.copy_(x)
                x = ax
                ao = arena_out[off:off + (out.numel() if out is not None else x.numel())]
                out = ao if out is not None else None
            stream.wait_stream(main)  # x and out were made on the main stream
            # NO host synchronisation between calls: consecutive calls on different streams must still be
            # serialised by the communicator (every collective shares the epochs and staging halves)
            with torch.cuda.stream(stream):
                busy = torch.randn(1 << 20, device="cuda").square_().sum()  # compute sharing the GPU
                calgo = "flat+zc" if zc else ("ring" if "ring" in spec else None)
                if coll == "allreduce":
                    y = comm.all_reduce(x, out=out, algo=spec)
                elif coll == "broadcast":
                    y = comm.broadcast(x, root=root, out=out, algo="flat+zc" if zc else None)
                elif coll == "all_to_all":
                    y = comm.all_to_all(x, out, algo="flat+zc" if zc else None)
                elif coll == "reduce_scatter":
                    y = comm.reduce_scatter(x, out, algo=calgo)
                else:
                    y = comm.all_gather(x, out, algo=calgo)
                if zc:
                    y = y.clone()  # the arenas are reused by later calls
            # keep x alive until the end: freed now, the caching allocator would hand its block to the next
            # iteration (main stream) while this call may still read it on the side stream
            pending.append((it, coll + ":" + spec, n, in_place, use_side, y, want, (x, busy)))
        torch.cuda.synchronize()
        for it, spec, n, in_place, use_side, y, want, _ in pending:
            if not torch.equal(y.cpu(), want):
                bad.append((it, spec, n, in_place, use_side))
        comm.check()
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, bad, None))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("world,fault", [(2, ""), (4, ""), (4, "delay:1:0:200")])
def test_ipc_randomized_call_sequence(cuda, world, fault):
    """Processes on one GPU run the same random sequence of collectives (allreduce with every algorithm,
    broadcast, all-to-all, reduce-scatter, all-gather), sizes, in/out-of-place and streams
    (with compute kernels sharing the GPU) with no host synchronisation between calls; every result is
    checked exactly (integer-valued fp32)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stress_worker, args=(r, world, port, 80, q, fault)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, bad, tb in res:
        assert tb is None, tb
        assert not bad, (rank, bad[:5])


def _readiness_worker(rank, world, port, q, fault):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000", FLEXAR_SELFTEST_TIMEOUT_MS="300")
        if fault.startswith("skew:"):
            os.environ["FLEXAR_SELFTEST_SKEW"] = fault[5:]
        elif fault.startswith("skewstrict:"):  # the one-GPU-per-rank policy, forced on the shared GPU
            os.environ["FLEXAR_SELFTEST_SKEW"] = fault[11:]
            os.environ["FLEXAR_SELFTEST_RETRY"] = "disable"
        elif fault:
            os.environ["FLEXAR_FAULT_INJECT"] = fault
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import Communicator

        comm = Communicator(workspace_bytes=32 << 20)
        topo = comm.topology()
        stats = comm.stats()
        # production calls after the gate: whatever family survived must give exact sums
        errs = {}
        for spec in ("flat+pull", "ring", "ll", "oneshot", None):
            x = torch.full((100003,), float(rank + 1), device="cuda")
            y = comm.all_reduce(x, algo=spec)
            torch.cuda.synchronize()
            errs[str(spec)] = (y - world * (world + 1) / 2).abs().max().item()
        desc = comm.describe(1 << 20, torch.float32)
        comm.check()
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, (topo, stats, errs, list(comm.selftest_failed), desc, list(comm.selftest_recovered)), None))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("fault", ["", "drop:1:0:0", "skew:1:1500", "skewstrict:1:1500"])
def test_ipc_connect_readiness_gate(cuda, fault):
    """Connect-time probe + exact self-test (readiness.hpp). Healthy: every family verified, peers on the
    same GPU. With rank 1 dropping its slot-0 SIGNAL (every executor schedule then breaks), the self-test
    disables the fence and write-through families on BOTH ranks and calls run on a verified family
    (copy engines / LL) with exact results instead of timing out. With rank 1 starting the first family
    1.5 s late (past the 0.3 s self-test watchdog: a transient failure), that family fails once, passes the
    repeat, and nothing is disabled."""
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_readiness_worker, args=(r, world, port, q, fault)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, out, tb in res:
        assert tb is None, tb
        topo, stats, errs, failed, desc, recovered = out
        assert [p["link"] for p in topo["peers"]] == ["self" if r == rank else "same-device" for r in range(world)]
        assert topo["peers"][rank]["bus"] and topo["links"] == 1
        assert stats["selftested"] == "fence,wt,ll,dma"
        assert stats["resident_blocks"] >= 256, stats
        if fault.startswith("skew:"):
            assert recovered == ["fence"] and failed == [] and stats["disabled"] == "", (recovered, failed, stats)
        elif fault.startswith("skewstrict:"):  # passed the repeat, disabled anyway
            assert recovered == [] and failed == ["fence"] and stats["disabled"] == "fence", (recovered, failed, stats)
        elif fault:
            assert failed == ["fence", "wt"], failed
            assert stats["disabled"] == "fence,wt"
            assert desc.startswith("dma"), desc
        else:
            assert failed == [] and stats["disabled"] == ""
        assert all(e == 0 for e in errs.values()), errs


def _zc_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000", FLEXAR_PROFILE="1")
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import Communicator

        comm = Communicator(workspace_bytes=32 << 20)
        dev = torch.device("cuda", 0)
        n = 1 << 20
        # two tensors carved out of one allocation (torch's allocator does this): one peer mapping serves both
        arena = torch.empty(2 * n + 64, device=dev)
        x, y = arena[:n], arena[n + 64:2 * n + 64]
        rx, ry = comm.register(x), comm.register(y)
        errs = {}
        for spec in ("flat+zc", "flat+zc+wt", "flat+zc+nts", "flat+zc+push", "flat+zc+push+wt", "flat+zc+put",
                     "flat+zc+put+wt", "flat+zc+put+nts"):
            for size in (7, 4096, 300001, n):
                for call in range(3):  # consecutive calls: a peer still reading the last call would show
                    src = torch.randn(size, generator=torch.Generator().manual_seed(1000 * rank + size + call))
                    x[:size].copy_(src.to(dev))
                    comm.all_reduce(x[:size], out=y[:size], algo=spec)
                    torch.cuda.synchronize()
                refs = [torch.randn(size, generator=torch.Generator().manual_seed(1000 * r + size + 2)) for r in range(world)]
                ref = torch.stack(refs).double().sum(0)
                errs[(spec, size)] = (y[:size].double().cpu() - ref).abs().max().item()
        # in place, at an offset inside the registration (the same offset on every rank)
        x[100:100 + 5003].fill_(float(rank + 1))
        comm.all_reduce(x[100:100 + 5003], algo="flat+zc")
        torch.cuda.synchronize()
        errs["in_place"] = (x[100:100 + 5003] - world * (world + 1) / 2).abs().max().item()
        x[100:100 + 5003].fill_(float(rank + 1))
        comm.all_reduce(x[100:100 + 5003], algo="flat+zc+push")
        torch.cuda.synchronize()
        errs["in_place_push"] = (x[100:100 + 5003] - world * (world + 1) / 2).abs().max().item()
        x[100:100 + 5003].fill_(float(rank + 1))
        comm.all_reduce(x[100:100 + 5003], algo="flat+zc+put")
        torch.cuda.synchronize()
        errs["in_place_put"] = (x[100:100 + 5003] - world * (world + 1) / 2).abs().max().item()
        # an unregistered buffer is refused, not read through a stale mapping
        try:
            comm.all_reduce(torch.ones(64, device=dev), algo="flat+zc")
            errs["unregistered"] = "accepted"
        except Exception as e:  # noqa: BLE001
            errs["unregistered"] = "refused" if "registered" in str(e) else str(e)
        # the other collectives: only the buffers a peer addresses need registering (reduce-scatter: the
        # inputs; all-gather / all-to-all / broadcast: the outputs)
        m = 70001
        big = torch.empty(3 * world * m + 128, device=dev)
        rs_in, ag_out, a2a_out = big[:world * m], big[world * m + 64:2 * world * m + 64], big[2 * world * m + 128:]
        regs = comm.register_many([rs_in, ag_out, a2a_out])  # one exchange for the three
        gen = torch.Generator().manual_seed(5)
        alls = [torch.randn(world * m, generator=gen) for _ in range(world)]
        rs_in.copy_(alls[rank].to(dev))
        total = torch.stack(alls).sum(0)
        for calgo in ("flat+zc", None):  # explicit, and the automatic switch on registered buffers
            rs_out = torch.empty(m, device=dev)
            comm.reduce_scatter(rs_in, rs_out, algo=calgo)
            ag_in = alls[rank][:m].to(dev)
            comm.all_gather(ag_in, ag_out, algo=calgo)
            comm.all_to_all(rs_in, a2a_out, algo=calgo)
            bsrc = alls[0][:m].to(dev) if rank == 0 else None
            comm.broadcast(bsrc if rank == 0 else ag_out[:m], root=0, out=ag_out[:m], algo="flat+zc")
            torch.cuda.synchronize()
            errs[f"rs_{calgo}"] = (rs_out.cpu() - total[rank * m:(rank + 1) * m]).abs().max().item()
            errs[f"a2a_{calgo}"] = (a2a_out.cpu() - torch.cat([alls[q][rank * m:(rank + 1) * m]
                                                               for q in range(world)])).abs().max().item()
            errs[f"ag_tail_{calgo}"] = (ag_out[m:].cpu() - torch.cat([alls[q][:m] for q in range(1, world)])).abs().max().item()
            errs[f"bcast_{calgo}"] = (ag_out[:m].cpu() - alls[0][:m]).abs().max().item()
        for rid in regs:
            comm.deregister(rid)
        # automatic choice (no spec): registered buffers run zero copy, unregistered ones the staging path,
        # and both give exact sums
        x.fill_(1.0)
        comm.all_reduce(x, out=y)
        z = torch.ones(n, device=dev)
        comm.all_reduce(z)
        torch.cuda.synchronize()
        errs["auto_registered"] = (y - world).abs().max().item()
        errs["auto_unregistered"] = (z - world).abs().max().item()
        prof = comm.stats()["profile"]
        errs["auto_used_zc"] = 0.0 if any("+zc" in k for k in prof) else 1.0
        errs["auto_used_staging"] = 0.0 if any("+zc" not in k for k in prof) else 1.0
        comm.deregister(rx)
        comm.deregister(ry)
        errs["regs_left"] = comm._lib.flexar_reg_count(comm._h)
        comm.check()
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, errs, None))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 4])
def test_ipc_zero_copy_registered_buffers(cuda, world):
    """"+zc": every rank reads its peers' registered input / output through IPC mappings (no staging)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_zc_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, errs, tb in res:
        assert tb is None, f"rank {rank} failed:\n{tb}"
        assert errs.pop("unregistered") == "refused"
        assert errs.pop("regs_left") == 0
        for key, err in errs.items():
            assert err < 1e-4, (rank, key, err)


@pytest.mark.skipif(not os.environ.get("FLEXAR_SOAK"), reason="soak run: FLEXAR_SOAK=<calls> (scripts/gpu_soak.sh)")
@pytest.mark.timeout(1000)
@pytest.mark.parametrize("world,fault", [(4, ""), (8, ""), (4, "delay:2:0:150")])
def test_ipc_soak(cuda, world, fault):
    """The randomized call sequence at length (FLEXAR_SOAK calls, e.g. 600): every collective, algorithm,
    size, stream and in/out-of-place mix, exact results, N = 4 and 8 on one GPU."""
    import torch.multiprocessing as mp

    if world > 4:
        os.environ["GPU_MAX_HW_QUEUES"] = "2"  # inherited by the spawned ranks
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    calls = int(os.environ["FLEXAR_SOAK"])
    procs = [ctx.Process(target=_stress_worker, args=(r, world, port, calls, q, fault)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=900) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, bad, tb in res:
        assert tb is None, tb
        assert not bad, (rank, len(bad), bad[:5])


def _rebuild_worker(rank, world, port, cycles, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000")
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import Communicator

        # the same buffers, registered by one communicator after another (what bench.py's fallback chain does
        # when it rebuilds): every cycle closes the communicator, with its IPC imports of the peers' buffers and
        # workspace, and maps the same allocations again in a fresh one
        n = 4 << 20
        x = torch.empty(n, device="cuda")
        y = torch.empty(n, device="cuda")
        bad = []
        for cyc in range(cycles):
            comm = Communicator(workspace_bytes=64 << 20)
            comm.register_many([x, y])
            for spec in ("flat+zc+push", "flat+zc", "flat+pull", "ll"):
                m = n if spec != "ll" else 4096
                x[:m].copy_(torch.arange(m, device="cuda", dtype=torch.float32) % 97 + rank + cyc)
                comm.all_reduce(x[:m], out=y[:m], algo=spec)
                torch.cuda.synchronize()
                want = (torch.arange(m, device="cuda", dtype=torch.float32) % 97) * world + world * (world - 1) / 2 \
                    + world * cyc
                if not torch.equal(y[:m], want):
                    bad.append((cyc, spec))
            comm.check()
            time.sleep(((rank * 7 + cyc * 3) % 5) * 0.006)  # ranks reach the collective teardown at different times
            comm.close()  # collective in the library: no caller barrier before the next communicator
        dist.destroy_process_group()
        q.put((rank, bad, None))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, None, traceback.format_exc()))


@pytest.mark.skipif(not os.environ.get("FLEXAR_SOAK"), reason="soak run: FLEXAR_SOAK (scripts/gpu_soak.sh)")
@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,cycles", [(2, 20), (4, 10)])
def test_ipc_communicator_rebuild_cycles(cuda, world, cycles):
    """Communicator rebuilds over the same registered buffers (close -> fresh communicator -> register the
    same allocations -> zero-copy and staging allreduces), ranks closing at staggered times with no caller
    barrier (the teardown agrees by itself), every result exact."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rebuild_worker, args=(r, world, port, cycles, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=500) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, bad, tb in res:
        assert tb is None, tb
        assert not bad, (rank, bad[:5])
