"""The "flexar" c10d backend + DDP on a real MI355X: two training processes on
one GPU (IPC between processes on one device), gradient allreduce through the
flexar executor kernel, compared against full-batch single-process training of
the same model. Also the DDP comm-hook path over a gloo process group.

The backend's default fallback group is RCCL (FLEXAR_PG_FALLBACK=nccl), which refuses two ranks on one GPU
of one host; the "+nccl" cases give every process its own NCCL_HOSTID so RCCL treats the ranks as separate
hosts (loopback sockets) and the production defaults run: RCCL fallback group, ProcessGroupNCCL cross-node
group of the hierarchical communicator, and DDP on the plain "nccl" backend as the reference trajectory."""
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


def _fallback_env(rank, fallback):
    """gloo fallback group, or RCCL's (the default) with one NCCL_HOSTID per rank on the shared GPU."""
    if fallback == "gloo":
        os.environ["FLEXAR_PG_FALLBACK"] = "gloo"
    else:
        os.environ.pop("FLEXAR_PG_FALLBACK", None)
        os.environ.update(NCCL_HOSTID=f"flexar-test-rank{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")


def _train(rank, world, port, q, mode, model_kind="mlp", fallback="gloo"):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000", FLEXAR_PG_ZC_MIN_BYTES="65536")  # GPT-tiny buckets register
        if mode == "backend_zcdefault":  # the backend's defaults: zero copy on (sweeps every 4 calls here)
            os.environ.pop("FLEXAR_PG_ZC", None)
            os.environ["FLEXAR_PG_ZC_SWEEP"] = "4"
            mode = "backend"
            steps, report_regs = 8, True
        elif mode == "backend_mx":  # the backend with FLEXAR_PG_COMPRESS: OCP MX fp8 gradients, no comm hook
            os.environ.update(FLEXAR_PG_COMPRESS="mx_e4m3", FLEXAR_PG_COMPRESS_MIN_BYTES="0", FLEXAR_PG_ZC="0")
            steps, report_regs = 4, False
        elif mode == "nccl8":  # the RCCL reference of the 8-step run above
            mode = "nccl"
            steps, report_regs = 8, False
        else:
            os.environ["FLEXAR_PG_ZC"] = "1"
            steps, report_regs = 4, False
        _fallback_env(rank, fallback)
        import torch.distributed as dist
        import torch.nn as nn
        from torch.nn.parallel import DistributedDataParallel as DDP

        from allreduce_over_mpi_amd.models.mlp import MLP
        from allreduce_over_mpi_amd.parallel import backend as fb

        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        pg_kind = {"backend": "flexar", "backend_mx": "flexar", "nccl": "nccl"}.get(mode, "gloo")
        if pg_kind == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(pg_kind, rank=rank, world_size=world)
        from allreduce_over_mpi_amd.models.gpt import GPT, PRESETS

        torch.manual_seed(0)
        make = (lambda: MLP()) if model_kind == "mlp" else (lambda: GPT(PRESETS["gpt-tiny"]))
        ref = make().to(dev)
        model = make().to(dev)
        model.load_state_dict(ref.state_dict())
        ddp = DDP(model, device_ids=[0], bucket_cap_mb=1)
        state = None
        if mode in ("hook", "fp8hook", "mxhook", "zchook"):
            # zchook: every gradient bucket registered on first sight, reduced by "flat+zc" (no staging)
            state = fb.FlexarHookState(zero_copy=mode == "zchook")
            ddp.register_comm_hook(state, {"fp8hook": fb.flexar_fp8_compress_hook,
                                           "mxhook": fb.flexar_mxfp8_compress_hook}.get(mode, fb.flexar_allreduce_hook))
        opt = torch.optim.SGD(ddp.parameters(), lr=0.05)
        ropt = torch.optim.SGD(ref.parameters(), lr=0.05)
        g = torch.Generator().manual_seed(42)
        def loss_fn(m, x, y):
            if model_kind == "mlp":
                return nn.functional.mse_loss(m(x), y)
            out = m(x)
            return nn.functional.cross_entropy(out.reshape(-1, out.shape[-1]), y.reshape(-1))

        for step in range(steps):
            if model_kind == "mlp":
                x = torch.randn(16 * world, 64, generator=g).to(dev)
                y = torch.randn(16 * world, 16, generator=g).to(dev)
            else:
                t = torch.randint(0, 512, (4 * world, 65), generator=g).to(dev)
                x, y = t[:, :-1], t[:, 1:]
            per = x.shape[0] // world
            sl = slice(rank * per, (rank + 1) * per)
            opt.zero_grad()
            loss_fn(ddp, x[sl], y[sl]).backward()
            opt.step()
            ropt.zero_grad()
            loss_fn(ref, x, y).backward()
            ropt.step()
        torch.cuda.synchronize()
        err = max((a - b).abs().max().item() for a, b in zip(model.parameters(), ref.parameters()))
        pg = dist.group.WORLD
        used = (getattr(pg, "stats", {}).get("flexar_allreduce", 0) if mode == "backend" else
                getattr(pg, "stats", {}).get("compressed", 0) if mode == "backend_mx" else
                1 if mode == "nccl" else state.calls)
        if mode == "backend" and model_kind == "gpt" and not pg.stats.get("zc_registrations"):
            used = 0  # the gradient buckets must have been registered (zero copy) by the backend's probe
        if mode == "zchook" and not state._bucket_regs:
            used = 0  # the zero-copy path must actually have registered the buckets
        if report_regs:
            pbytes = sum(p.numel() * p.element_size() for p in model.parameters())
            used = {"calls": used, "registered_bytes": pg.zc_registered_bytes(), "param_bytes": pbytes,
                    "registrations": pg.stats.get("zc_registrations", 0),
                    "deregistrations": pg.stats.get("zc_deregistrations", 0)}
        dist.destroy_process_group()
        # numpy arrays travel by value (a torch CPU tensor would be shared through a descriptor of this exiting process)
        q.put((rank, err, used, None, [p.detach().cpu().numpy() for p in model.parameters()]))
    except Exception:
        import traceback

        q.put((rank, None, None, traceback.format_exc(), None))


def _spawn(target, world, *args, timeout=300):
    """Run ``target(rank, world, port, q, *args)`` in ``world`` spawned processes; the results by rank.
    A rank that hangs is killed (it must not outlive the test on the GPU)."""
    import queue

    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=target, args=(r, world, port, q, *args)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = [q.get(timeout=timeout) for _ in range(world)]
    except queue.Empty:
        pytest.fail(f"{target.__name__}: a rank did not finish within {timeout} s")
    finally:
        for p in ps:
            p.join(60)
            if p.is_alive():
                p.kill()
    return res


@pytest.mark.parametrize("mode,model_kind,fallback", [
    ("backend", "mlp", "gloo"), ("hook", "mlp", "gloo"), ("backend", "gpt", "gloo"), ("hook", "gpt", "gloo"),
    ("fp8hook", "mlp", "gloo"), ("mxhook", "mlp", "gloo"), ("backend_mx", "mlp", "gloo"), ("zchook", "mlp", "gloo"), ("zchook", "gpt", "gloo"), ("backend", "gpt", "nccl")])
def test_ddp_over_flexar(cuda, mode, model_kind, fallback):
    res = _spawn(_train, 2, mode, model_kind, fallback)
    for rank, err, used, tb, _ in res:
        assert tb is None, tb
        assert used and used > 0, "flexar path was not used"
        # fp8 on the wire: e4m3's 2^-4 relative step of each bucket's largest gradient, over 4 SGD steps
        tol = 1e-2 if mode in ("fp8hook", "mxhook", "backend_mx") else (1e-5 if model_kind == "mlp" else 2e-4)
        assert err < tol, (mode, model_kind, rank, err)


def test_ddp_flexar_backend_matches_rccl_ddp(cuda):
    """SURVEY.md section 7.4's criterion: DDP on the "flexar" backend (default RCCL fallback group) follows the
    same trajectory as DDP on the plain "nccl" backend. Two ranks: every gradient element is a sum of two
    addends, the same in any order, so the parameters agree exactly."""
    ours = {r: params for r, _, _, tb, params in _spawn(_train, 2, "backend", "gpt", "nccl") if tb is None}
    rccl = {r: params for r, _, _, tb, params in _spawn(_train, 2, "nccl", "gpt", "nccl") if tb is None}
    assert len(ours) == 2 and len(rccl) == 2
    for r in range(2):
        for a, b in zip(ours[r], rccl[r]):
            assert (a == b).all(), (r, abs(a - b).max())


def test_backend_zero_copy_default_stays_bounded(cuda):
    """init_process_group("flexar") with the defaults (zero copy on): DDP's gradient
    buckets are registered, DDP's bucket rebuild after the first iteration leaves the first buckets to the
    registrations alone, and the collective sweep frees them - the registered bytes stay within one set of
    buckets - while training stays bit-identical to DDP over RCCL."""
    ours = _spawn(_train, 2, "backend_zcdefault", "gpt", "nccl")
    rccl = {r: params for r, _, _, tb, params in _spawn(_train, 2, "nccl8", "gpt", "nccl") if tb is None}
    for rank, err, info, tb, params in ours:
        assert tb is None, tb
        assert info["calls"] > 0 and info["registrations"] > 0, info
        # one bucket set: at most the gradients' bytes (+ one bucket of rounding), never both sets pinned
        assert info["registered_bytes"] <= info["param_bytes"] + (1 << 20), info
        assert info["deregistrations"] > 0, info  # DDP's first bucket set was freed after its rebuild
        for a, b in zip(params, rccl[rank]):
            assert (a == b).all(), (rank, abs(a - b).max())


def _colls(rank, world, port, q, fallback="gloo"):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000")
        _fallback_env(rank, fallback)
        import torch.distributed as dist

        from allreduce_over_mpi_amd.parallel import backend as fb  # noqa: F401

        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("flexar", rank=rank, world_size=world)
        m = 1001
        full = torch.arange(world * m, dtype=torch.float32, device=dev) * (rank + 1)
        out = torch.empty(m, device=dev)
        dist.reduce_scatter_tensor(out, full)
        want = torch.arange(world * m, dtype=torch.float32, device=dev)[rank * m:(rank + 1) * m] * sum(
            r + 1 for r in range(world))
        e1 = (out - want).abs().max().item()
        part = torch.full((m,), float(rank), device=dev)
        gat = torch.empty(world * m, device=dev)
        dist.all_gather_into_tensor(gat, part)
        e2 = (gat - torch.arange(world, device=dev).float().repeat_interleave(m)).abs().max().item()
        x = torch.ones(5, device=dev)
        dist.all_reduce(x, op=dist.ReduceOp.AVG)
        e3 = (x - 1).abs().max().item()
        # list forms (dist.all_gather / dist.reduce_scatter) and the coalesced tensor forms FSDP2 issues
        outs = [torch.empty(7, 3, device=dev) for _ in range(world)]
        dist.all_gather(outs, torch.full((7, 3), float(rank + 1), device=dev))
        e4 = max((o - (r + 1)).abs().max().item() for r, o in enumerate(outs))
        chunks = [torch.full((9,), float((rank + 1) * (c + 1)), device=dev) for c in range(world)]
        rs = torch.empty(9, device=dev)
        dist.reduce_scatter(rs, chunks)
        e5 = (rs - (rank + 1) * sum(r + 1 for r in range(world))).abs().max().item()
        pg = dist.group.WORLD
        ins = [torch.full((m,), float(rank), device=dev), torch.full((3,), float(rank) + 0.5, device=dev)]
        gos = [torch.empty(world * m, device=dev), torch.empty(world * 3, device=dev)]
        pg.allgather_into_tensor_coalesced(gos, ins).wait()
        e6 = max((gos[0] - torch.arange(world, device=dev).float().repeat_interleave(m)).abs().max().item(),
                 (gos[1] - (torch.arange(world, device=dev).float() + 0.5).repeat_interleave(3)).abs().max().item())
        rsi = [torch.ones(world * 4, device=dev) * (rank + 1), torch.ones(world * 2, device=dev)]
        rso = [torch.empty(4, device=dev), torch.empty(2, device=dev)]
        pg.reduce_scatter_tensor_coalesced(rso, rsi).wait()
        e7 = max((rso[0] - sum(r + 1 for r in range(world))).abs().max().item(), (rso[1] - world).abs().max().item())
        a2i = torch.arange(world * 5, device=dev, dtype=torch.float32) + 100 * rank
        a2o = torch.empty_like(a2i)
        dist.all_to_all_single(a2o, a2i)
        want_a2 = torch.cat([torch.arange(rank * 5, rank * 5 + 5, device=dev).float() + 100 * r for r in range(world)])
        e9 = (a2o - want_a2).abs().max().item()
        bc = torch.arange(100003, device=dev, dtype=torch.float32) * (rank + 1)
        dist.broadcast(bc, src=1)
        e8 = (bc - torch.arange(100003, device=dev).float() * 2).abs().max().item()
        # list-form all-to-all (packed into one flexar exchange)
        a2l_in = [torch.full((2, 3), float(10 * rank + p), device=dev) for p in range(world)]
        a2l_out = [torch.empty(2, 3, device=dev) for _ in range(world)]
        dist.all_to_all(a2l_out, a2l_in)
        e12 = max((o - float(10 * p + rank)).abs().max().item() for p, o in enumerate(a2l_out))
        # dist.reduce: the root gets the sum, every other rank's tensor stays as it was
        rd = torch.arange(70001, device=dev, dtype=torch.float32) * (rank + 1)
        dist.reduce(rd, dst=world - 1)
        k = sum(r + 1 for r in range(world)) if rank == world - 1 else rank + 1
        e11 = (rd - torch.arange(70001, device=dev).float() * k).abs().max().item()
        # dist.reduce on a tensor the zero-copy probe registered: the root must not pick the
        # registered-buffer schedule while the other ranks stage (that mismatch hangs until the watchdog)
        big = torch.full((1 << 19,), float(rank + 1), device=dev)  # 2 MiB: above FLEXAR_PG_ZC_MIN_BYTES
        for _ in range(3):
            dist.all_reduce(big)
            big.fill_(float(rank + 1))
        registered = dist.group.WORLD.stats.get("zc_registrations", 0)
        dist.reduce(big, dst=0)
        k2 = sum(r + 1 for r in range(world)) if rank == 0 else rank + 1
        e13 = (big - k2).abs().max().item() if registered else 1.0
        torch.cuda.synchronize()
        e10 = 0.0
        if fallback == "nccl":  # point-to-point (pipeline stages) has no flexar program: RCCL by default
            pp = torch.full((4099,), float(rank + 1), device=dev)
            if rank == 0:
                dist.send(pp, dst=1)
            elif rank == 1:
                dist.recv(pp, src=0)
            e10 = (pp - (1.0 if rank <= 1 else rank + 1.0)).abs().max().item()
            e10 = e10 if dist.group.WORLD.stats["fallback"] > 0 else 1.0
        dist.barrier()
        used = dist.group.WORLD.stats["flexar_allreduce"]
        dist.destroy_process_group()
        q.put((rank, max(e1, e2, e3, e4, e5, e6, e7, e8, e9, e10, e11, e12, e13), used, None))
    except Exception:
        import traceback

        q.put((rank, None, None, traceback.format_exc()))


@pytest.mark.parametrize("fallback", ["gloo", "nccl"])
def test_backend_reduce_scatter_all_gather(cuda, fallback):
    for rank, err, used, tb in _spawn(_colls, 2, fallback):
        assert tb is None, tb
        assert err == 0.0 and used >= 11, (rank, err, used)


def test_rccl_algo_routing_single_rank():
    """algo="rccl" / FLEXAR_ALGO=rccl routes Communicator.all_reduce to RCCL (one rank: RCCL refuses two
    ranks on one GPU)."""
    import subprocess
    import sys

    code = r'''
import os, torch, torch.distributed as dist
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ["PORT"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1)
from allreduce_over_mpi_amd.parallel import Communicator
c = Communicator()
x = torch.arange(1000, device="cuda", dtype=torch.float32)
y = torch.empty_like(x)
c.all_reduce(x, out=y, algo="rccl", scale=0.5)
assert torch.equal(y, x * 0.5)
c.set_algo("rccl")
z = x.clone()
c.all_reduce(z, op="max")
assert torch.equal(z, x)
c.set_algo("flat")
c.all_reduce(z)
assert torch.equal(z, x)
c.close()
dist.destroy_process_group()
print("rccl routing ok")
'''
    env = dict(os.environ, PORT=str(_port()), PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "rccl routing ok" in r.stdout, r.stdout + r.stderr


def _hier_backend(rank, world, port, q, fallback="gloo"):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000", FLEXAR_NODE_SIZE="2")
        _fallback_env(rank, fallback)
        import torch.distributed as dist

        from allreduce_over_mpi_amd.parallel import backend as fb  # noqa: F401

        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("flexar", rank=rank, world_size=world)
        errs = []
        for n in (1, 7, 100003):
            x = torch.arange(n, device=dev, dtype=torch.float32) + rank
            dist.all_reduce(x)
            want = torch.arange(n, device=dev).float() * world + sum(range(world))
            errs.append((x - want).abs().max().item())
            y = torch.full((n,), float(rank + 1), device=dev)
            dist.all_reduce(y, op=dist.ReduceOp.MAX)
            errs.append((y - world).abs().max().item())
        b = torch.full((33,), float(rank), device=dev)
        dist.broadcast(b, src=3)  # hierarchical communicator: broadcast takes the fallback group
        errs.append((b - 3).abs().max().item())
        pg = dist.group.WORLD
        ok = pg.hierarchical and pg.stats["flexar_allreduce"] >= 6 and pg.stats["fallback"] >= 1
        dist.destroy_process_group()
        q.put((rank, max(errs), ok, None))
    except Exception:
        import traceback

        q.put((rank, None, None, traceback.format_exc()))


@pytest.mark.parametrize("fallback", ["gloo", "nccl"])
def test_backend_hierarchical_virtual_nodes(cuda, fallback):
    """init_process_group("flexar") over 2 virtual nodes x 2 ranks: dist.all_reduce runs intra-node flexar
    reduce-scatter / all-gather around a cross-node allreduce of the shards ("nccl": the production
    ProcessGroupNCCL cross-node group, one NCCL_HOSTID per rank)."""
    for rank, err, ok, tb in _spawn(_hier_backend, 4, fallback):
        assert tb is None, tb
        assert err == 0.0 and ok, (rank, err, ok)


def _hier_backend_mx(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000", FLEXAR_NODE_SIZE="2", FLEXAR_PG_FALLBACK="gloo",
                          FLEXAR_PG_COMPRESS="mx_e4m3", FLEXAR_PG_COMPRESS_MIN_BYTES="65536")
        import torch.distributed as dist

        from allreduce_over_mpi_amd.ops.quant import mx_round
        from allreduce_over_mpi_amd.parallel import backend as fb  # noqa: F401

        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("flexar", rank=rank, world_size=world)
        n = 100002
        xs = [torch.randn(n, generator=torch.Generator().manual_seed(7 + r)) for r in range(world)]
        m = n // 2
        want = torch.empty(n)
        for l in range(2):  # exact node pairs, MX per node shard, node order
            sl = slice(l * m, (l + 1) * m)
            want[sl] = mx_round(xs[0][sl] + xs[1][sl]) + mx_round(xs[2][sl] + xs[3][sl])
        x = xs[rank].to(dev)
        dist.all_reduce(x)  # 400 KB >= the 64 KiB threshold: compressed across nodes
        small = torch.full((1000,), float(rank), device=dev)
        dist.all_reduce(small)  # under the threshold: exact
        pg = dist.group.WORLD
        res = (int((x.cpu() != want).sum()), (small - 6).abs().max().item(), pg.stats.get("compressed", 0))
        dist.destroy_process_group()
        q.put((rank, res, None))
    except Exception:
        import traceback

        q.put((rank, None, traceback.format_exc()))


def test_backend_hierarchical_compressed(cuda):
    """FLEXAR_NODE_SIZE=2 + FLEXAR_PG_COMPRESS=mx_e4m3: dist.all_reduce keeps the intra-node steps exact and
    carries OCP MX fp8 across the (virtual) nodes - bitwise the torch reference; calls under the threshold
    stay exact."""
    for rank, res, tb in _spawn(_hier_backend_mx, 4):
        assert tb is None, tb
        mism, small_err, compressed = res
        assert mism == 0 and small_err == 0.0 and compressed == 1, (rank, res)


def _fsdp_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_PG_FALLBACK="gloo", FLEXAR_TIMEOUT_MS="20000")
        import torch.distributed as dist
        import torch.nn as nn
        from torch.distributed.device_mesh import init_device_mesh
        from torch.distributed.fsdp import fully_shard

        from allreduce_over_mpi_amd.models.mlp import MLP
        from allreduce_over_mpi_amd.parallel import backend as fb  # noqa: F401

        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("flexar", rank=rank, world_size=world)
        mesh = init_device_mesh("cuda", (world,))
        torch.manual_seed(0)
        ref = MLP().to(dev)
        model = MLP().to(dev)
        model.load_state_dict(ref.state_dict())
        for layer in model.net:
            if isinstance(layer, nn.Linear):
                fully_shard(layer, mesh=mesh)
        fully_shard(model, mesh=mesh)
        opt = torch.optim.SGD(model.parameters(), lr=0.05)
        ropt = torch.optim.SGD(ref.parameters(), lr=0.05)
        g = torch.Generator().manual_seed(7)
        for _ in range(3):
            x = torch.randn(16 * world, 64, generator=g).to(dev)
            y = torch.randn(16 * world, 16, generator=g).to(dev)
            sl = slice(rank * 16, (rank + 1) * 16)
            opt.zero_grad()
            nn.functional.mse_loss(model(x[sl]), y[sl]).backward()
            opt.step()
            ropt.zero_grad()
            nn.functional.mse_loss(ref(x), y).backward()
            ropt.step()
        torch.cuda.synchronize()
        full = {k: v.full_tensor() for k, v in model.state_dict().items()}
        err = max((full[k] - v).abs().max().item() for k, v in ref.state_dict().items())
        used = dist.group.WORLD.stats["flexar_allreduce"]
        dist.destroy_process_group()
        q.put((rank, err, used, None))
    except Exception:
        import traceback

        q.put((rank, None, None, traceback.format_exc()))


def test_fsdp2_over_flexar(cuda):
    """FSDP2 (fully_shard) on the "flexar" backend: parameter all-gathers and gradient reduce-scatters run the
    flexar programs; 3 SGD steps match full-batch single-process training."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_fsdp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in ps:
        p.join(60)
    for rank, err, used, tb in res:
        assert tb is None, tb
        assert used and used > 0, "flexar collectives were not used"
        assert err < 1e-5, (rank, err)


def _funcol(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000")
        _fallback_env(rank, "gloo")
        import torch.distributed as dist
        import torch.distributed._functional_collectives as funcol

        from allreduce_over_mpi_amd.parallel import backend as fb  # noqa: F401

        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("flexar", rank=rank, world_size=world)
        tri = sum(r + 1 for r in range(world))
        # the functional collectives (DTensor / tensor parallelism, torch.compile-traceable): all_reduce,
        # reduce_scatter_tensor and all_gather_tensor through the "flexar" process group
        a = funcol.wait_tensor(funcol.all_reduce(torch.full((4099,), float(rank + 1), device=dev), "sum",
                                                 dist.group.WORLD))
        rs = funcol.wait_tensor(funcol.reduce_scatter_tensor(
            torch.arange(world * 1000, device=dev, dtype=torch.float32) * (rank + 1), "sum", 0, dist.group.WORLD))
        ag = funcol.wait_tensor(funcol.all_gather_tensor(torch.full((513,), float(rank), device=dev), 0,
                                                         dist.group.WORLD))
        torch.cuda.synchronize()
        err = max((a - tri).abs().max().item(),
                  (rs - torch.arange(rank * 1000, (rank + 1) * 1000, device=dev).float() * tri).abs().max().item(),
                  (ag - torch.arange(world, device=dev).float().repeat_interleave(513)).abs().max().item())
        used = dist.group.WORLD.stats["flexar_allreduce"]
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, err, used, None))
    except Exception:
        import traceback

        q.put((rank, None, None, traceback.format_exc()))


def test_functional_collectives_over_flexar(cuda):
    """torch.distributed._functional_collectives (what DTensor, tensor parallelism and torch.compile issue)
    dispatch into the "flexar" backend's allreduce / reduce-scatter / all-gather."""
    for rank, err, used, tb in _spawn(_funcol, 2):
        assert tb is None, tb
        assert err == 0.0 and used >= 3, (rank, err, used)


def _compressed_rs(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16", FLEXAR_PG_ZC="0",
                          FLEXAR_PG_COMPRESS="mx_e4m3", FLEXAR_PG_COMPRESS_MIN_BYTES="0")
        _fallback_env(rank, "gloo")
        import torch.distributed as dist

        import allreduce_over_mpi_amd.parallel.backend  # noqa: F401  registers "flexar"
        from allreduce_over_mpi_amd.ops.quant import mx_reduce_scatter_reference

        torch.cuda.set_device(0)
        dist.init_process_group("flexar", rank=rank, world_size=world)
        m = 65537
        xs = [torch.randn(world * m, generator=torch.Generator().manual_seed(50 + r)) for r in range(world)]
        out = torch.empty(m, device="cuda")
        dist.reduce_scatter_tensor(out, xs[rank].cuda(), op=dist.ReduceOp.AVG)
        torch.cuda.synchronize()
        want = mx_reduce_scatter_reference(xs, "e4m3", "avg")[rank]
        bad = int((out.cpu().view(torch.uint8) != want.view(torch.uint8)).sum())
        stats = dict(dist.group.WORLD.stats)
        dist.destroy_process_group()
        q.put((rank, bad, stats, None))
    except Exception:
        import traceback

        q.put((rank, None, None, traceback.format_exc()))


def test_backend_compressed_reduce_scatter(cuda):
    """FLEXAR_PG_COMPRESS=mx_e4m3: the backend's reduce_scatter_tensor (FSDP's gradient path) runs the flat
    reduce-scatter with the OCP MX wire, byte for byte the reference arithmetic."""
    for rank, bad, stats, tb in _spawn(_compressed_rs, 2):
        assert tb is None, tb
        assert bad == 0, (rank, bad)
