"""The xGMI acceptance matrix, runnable on every box.

One process per rank, workspaces mapped through HIP IPC, bootstrap through torch.distributed (gloo), RCCL
message transport next to it. The device map is a parameter: with at least N GPUs every rank gets its own
device (the production topology: peers over xGMI); on a 1-GPU box every rank uses device 0 (same handle
exchange, mappings and system-scope flag protocol, one HBM). The body is identical either way, so the
first multi-GPU GPUTEST runs exactly what every 1-GPU GPUTEST already ran.

Matrix (every result against a float64 host reference; inputs x, x/2, x/4 on alternating staging
parities, so a stale staging line cannot go unnoticed):
* allreduce: flat / ring / oneshot / ll / dma / bidir / +rccl, the FlexTree family (mixed-radix trees
  2,4 and 4,2 at N = 8 - 2,2 at N = 4 - with push and pull all-gather, RHD), multi-channel rings, fp32 and
  bf16, SUM and the fused AVG, uneven tail sizes, in place;
* typed bf16 partials ("+f32", one rounding) and per-hop rounding ("+rw") of the multi-hop schedules;
* all_reduce_fp8 (fused pre/post-scale, e4m3 wire) against a torch emulation of the same arithmetic, and the
  OCP MX wire ("flat+mxe4m3", block scales, no amax pass) bit for bit against ops.quant.mx_allreduce_reference;
* reduce-scatter / all-gather / all-to-all / broadcast (staging and zero copy);
* zero-copy allreduce over registered buffers;
* executor grid requests of 256, 512 and 1024 workgroups when ranks do not share a device (clamped to
  the resident workgroups);
* DDP GPT-tiny over a "flexar" process group against one model trained on the whole batch.
"""
import os
import socket
import sys

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


def _specs(world):
    specs = ["flat", "flat+push", "flat+wt", "flat+push+nts", "ring", "ring+wt", "oneshot", "ll", "dma", "flat+bidir",
             "flat+rccl", "ring+rccl"]
    from allreduce_over_mpi_amd import _native as nv

    chans = len([d for d in range(1, world) if __import__("math").gcd(d, world) == 1])
    specs += [f"ring:{c}" for c in (2, 4) if c <= chans]
    full = nv.ring_order(world, 0, 1)[1]  # N - 1 arc-disjoint rings over the full mesh (ring:7 at N = 8)
    if full > max(4, chans):
        specs.append(f"ring:{full}")
    if world == 4:
        specs += ["tree:2,2+push", "tree:2,2+pull", "tree:2,2+push+wt", "rhd+rccl", "rhd:3+pull", "rhd:3+push"]
    if world == 8:
        specs += ["tree:2,4+push", "tree:2,4+pull", "tree:4,2+push", "tree:4,2+pull", "rhd", "rhd+rccl",
                  "rhd:7+pull", "rhd:7+push", "tree:4,2:7+pull", "tree:2,4:7+push+nts"]
    if world in (3, 6):
        specs += [f"tree:{a},{b}+pull" for a, b in ((2, world // 2),) if a * b == world]
    assert all(nv.model_cost_us(s.replace("+rccl", ""), world, 1e6) > 0 for s in specs)
    return specs


def _typed_specs(world):
    out = ["ring+f32", "ring+rw"]
    if world >= 4 and not world & (world - 1):
        out += ["rhd+pull+f32", "rhd+pull+rw", f"rhd:{world - 1}+pull+f32", f"rhd:{world - 1}+pull+rw"]
    if world == 8:
        out += ["tree:4,2+pull+f32", "tree:4,2+pull+rw"]
    return out


def _emulate_fp8_flat(xs, s, op):
    """Torch emulation of flat+pull over an e4m3 wire (device_exec.hpp typed XFERs): each contribution
    quantised once with the pre-scale s, the owner sums in fp32 (rank order from the owner), the result is
    quantised once for the all-gather and every rank writes q / s in the buffer's dtype."""
    wire = torch.float8_e4m3fn
    n = len(xs)
    q = [(x.float() * s).to(wire).float() for x in xs]
    count = xs[0].numel()
    split = -(-count // n)
    split = -(-split // 256) * 256
    out = torch.empty(count)
    for k in range(n):
        lo, hi = k * split, min(count, (k + 1) * split)
        if lo >= hi:
            continue
        acc = q[k][lo:hi].clone()
        for jj in range(1, n):
            acc = acc + q[(k + jj) % n][lo:hi]
        if op == "avg":
            acc = acc * (1.0 / n)
        out[lo:hi] = acc.to(wire).float()
    return (out * (1.0 / s)).to(xs[0].dtype)


def _worker(rank, world, port, shared, q, transport="rccl", no_ipc=False, parts=("all",)):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_TIMEOUT_MS="20000")
        if shared:  # every rank on device 0: co-resident grids, one NCCL_HOSTID per rank (RCCL over loopback)
            os.environ.update(FLEXAR_MAX_GRID=str(max(8, 256 // (2 * world))), NCCL_HOSTID=f"flexar-md-rank{rank}",
                              NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
            # 8 processes x 4 hardware queues would be time-sliced by the command processor; a cap, since the
            # GPU box exports HIP's default of 4 explicitly
            if world > 4 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) > 2:
                os.environ["GPU_MAX_HW_QUEUES"] = "2"
        if no_ipc:
            os.environ["FLEXAR_FAULT_NO_IPC"] = "1"  # every peer mapping fails: the RCCL fallback carries all
        import torch.distributed as dist

        d = 0 if shared else rank
        torch.cuda.set_device(d)
        dev = torch.device("cuda", d)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd.parallel import Communicator

        comm = Communicator(workspace_bytes=128 << 20, transport=transport)
        results = {}
        big = 262147 if shared else 1000003

        def inputs(size, seed, dtype):
            return [torch.randn(size, generator=torch.Generator().manual_seed(seed * 131 + r + size)).to(dtype)
                    for r in range(world)]

        def rel(y, want):
            return ((y.double().cpu() - want).abs().max() / (want.abs().max() + 1e-12)).item()

        def allreduce_case(spec, dtype, sizes, ops=("sum", "avg"), in_place=False):
            print(f"[rank {rank}] allreduce {spec} {dtype} {sizes} in_place={in_place}", file=sys.stderr, flush=True)
            for size in sizes:
                xs = inputs(size, 1, dtype)
                ref = torch.stack([x.double() for x in xs]).sum(0)
                for op in ops:
                    worst = 0.0
                    for s in (1.0, 0.5, 0.25):
                        x = (xs[rank].double() * s).to(dtype).to(dev)
                        y = comm.all_reduce(x, op=op, algo=spec) if in_place else \
                            comm.all_reduce(x, op=op, algo=spec, out=torch.empty_like(x))
                        torch.cuda.synchronize()
                        worst = max(worst, rel(y, ref * s / (world if op == "avg" else 1)))
                    results[("allreduce", spec, str(dtype), size, op, in_place)] = worst

        if "all" in parts or "allreduce" in parts:
            for spec in _specs(world) if not no_ipc else ["flat", "ring", "oneshot"] + (
                    ["rhd", "tree:2,2"] if world == 4 else []):
                for dtype in (torch.float32, torch.bfloat16):
                    allreduce_case(spec, dtype, (5, 4096, big))
            for spec in ("flat", "ring", "oneshot") + (("rhd",) if world >= 4 and not world & (world - 1) else ()):
                allreduce_case(spec, torch.float32, (4097, big), ops=("sum",), in_place=True)
        if no_ipc:
            parts = ()
        if "all" in parts or "typed" in parts:
            for spec in _typed_specs(world):
                allreduce_case(spec, torch.bfloat16, (4096, big), ops=("sum",))
        if "all" in parts or "fp8" in parts:
            for dtype, op in ((torch.float32, "avg"), (torch.bfloat16, "avg"), (torch.float32, "sum")):
                xs = [x * (r + 1) for r, x in enumerate(inputs(big, 5, dtype))]
                amax = max(float(x.float().abs().max()) for x in xs)
                from allreduce_over_mpi_amd.ops.quant import fp8_wire_scale

                s = fp8_wire_scale(world, amax)  # the device's pre-scale (device_exec.hpp fp8_scale)
                want = _emulate_fp8_flat(xs, s, op)
                ref = torch.stack([x.double() for x in xs]).sum(0) / (world if op == "avg" else 1)
                for _ in range(3):
                    y = comm.all_reduce_fp8(xs[rank].to(dev), op=op)
                    torch.cuda.synchronize()
                mism = (~torch.isclose(y.float().cpu(), want.float(), rtol=1e-5, atol=0)).float().mean().item()
                results[("fp8_emulation_mismatch", str(dtype), op)] = mism
                results[("fp8_rel", str(dtype), op)] = rel(y, ref)
            # OCP MX wire (block scales, no amax pass): bit for bit the reference arithmetic
            from allreduce_over_mpi_amd.ops.quant import mx_allreduce_reference

            for dtype, spec in ((torch.float32, "flat+mxe4m3"), (torch.bfloat16, "flat+mxe4m3"),
                                (torch.bfloat16, "flat+wt+mxe5m2")):
                xs = [x * (r + 1) for r, x in enumerate(inputs(big, 9, dtype))]
                want = mx_allreduce_reference(xs, spec.rsplit("+mx", 1)[1], "avg")
                for _ in range(3):
                    y = comm.all_reduce(xs[rank].to(dev), op="avg", algo=spec)
                    torch.cuda.synchronize()
                results[("mx_mismatch", str(dtype), spec)] = int((y.cpu().view(torch.uint8) != want.view(torch.uint8)).sum())
            from allreduce_over_mpi_amd.ops.quant import mx_reduce_scatter_reference

            m = 100003
            xs = inputs(world * m, 11, torch.bfloat16)
            want = mx_reduce_scatter_reference(xs, "e4m3", "avg")[rank]
            out = torch.empty(m, device=dev, dtype=torch.bfloat16)
            for _ in range(2):
                comm.reduce_scatter(xs[rank].to(dev), out, op="avg", algo="flat+mxe4m3")
                torch.cuda.synchronize()
            results[("mx_mismatch", "rs", "flat+mxe4m3")] = int((out.cpu().view(torch.uint8) != want.view(torch.uint8)).sum())
        if "all" in parts or "colls" in parts:
            m = 4099
            for spec in (None, "ring", "flat+wt"):
                xs = inputs(world * m, 7, torch.float32)
                ref = torch.stack([x.double() for x in xs]).sum(0)
                out = torch.empty(m, device=dev)
                comm.reduce_scatter(xs[rank].to(dev), out, algo=spec)
                torch.cuda.synchronize()
                results[("reduce_scatter", spec)] = rel(out, ref[rank * m:(rank + 1) * m])
                ins = inputs(m, 8, torch.float32)
                full = torch.empty(world * m, device=dev)
                comm.all_gather(ins[rank].to(dev), full, algo=spec)
                torch.cuda.synchronize()
                results[("all_gather", spec)] = rel(full, torch.cat(ins).double())
            a2a_in = inputs(world * m, 9, torch.float32)
            a2a_out = torch.empty(world * m, device=dev)
            comm.all_to_all(a2a_in[rank].to(dev), a2a_out)
            torch.cuda.synchronize()
            want = torch.cat([a2a_in[p][rank * m:(rank + 1) * m] for p in range(world)]).double()
            results[("all_to_all", None)] = rel(a2a_out, want)
            for root in (0, world - 1):
                for spec in (None, "oneshot", "flat"):
                    src = inputs(big, 10 + root, torch.float32)[root]
                    t = (src if rank == root else torch.zeros_like(src)).to(dev)
                    comm.broadcast(t, root=root, algo=spec)
                    torch.cuda.synchronize()
                    results[("broadcast", root, spec)] = rel(t, src.double())
        if "all" in parts or "zc" in parts:
            for dtype in (torch.float32, torch.bfloat16):
                arena = torch.empty(1000003, device=dev, dtype=dtype)
                out = torch.empty_like(arena)
                comm.register_many([arena, out])
                for spec in ("flat+zc", "flat+zc+push", "flat+zc+push+wt", "flat+zc+put", "flat+zc+put+nts"):
                    for size in (5, 4096, 1000003):
                        xs = inputs(size, 11, dtype)
                        ref = torch.stack([x.double() for x in xs]).sum(0)
                        for call in range(3):  # consecutive calls: the closing hand-off
                            arena[:size].copy_(xs[rank].to(dev))
                            comm.all_reduce(arena[:size], out=out[:size], algo=spec)
                        torch.cuda.synchronize()
                        results[("zc", spec, str(dtype), size)] = rel(out[:size], ref)
            # zero-copy reduce-scatter / all-gather over registered buffers
            m = 8191
            rs_in = torch.empty(world * m, device=dev)
            rs_out = torch.empty(m, device=dev)
            comm.register_many([rs_in, rs_out])
            xs = inputs(world * m, 12, torch.float32)
            rs_in.copy_(xs[rank].to(dev))
            comm.reduce_scatter(rs_in, rs_out, algo="flat+zc")
            torch.cuda.synchronize()
            ref = torch.stack([x.double() for x in xs]).sum(0)
            results[("zc_reduce_scatter", None)] = rel(rs_out, ref[rank * m:(rank + 1) * m])
        if ("all" in parts or "grids" in parts) and not shared:
            # grids from 256 up to past residency: a request beyond the workgroups the GPU keeps resident is
            # clamped to them (comm.hip choose_grid), so the flag protocol never depends on dispatch order
            resident = int(comm.topology()["resident_blocks"])
            for g in (256, 512, 1024):
                comm.set_grid(g)
                for spec in ("flat", "flat+push+nts", "ring"):
                    allreduce_case(spec, torch.float32, (1 << 22,), ops=("sum",))
                    results[("grid", g, spec)] = results.pop(("allreduce", spec, str(torch.float32), 1 << 22, "sum",
                                                              False))
                used = int(comm.describe(1 << 22, torch.float32).split("grid=")[1].split()[0])
                results[("grid_clamped", g)] = 0.0 if used <= max(resident, 1) else float(used)
            comm.set_grid(0)
        comm.check()
        results["readiness"] = (comm.topology(), list(comm.selftest_failed))
        comm.close()
        if "all" in parts or "ddp" in parts:
            results[("ddp", "gpt-tiny")] = _ddp_gpt(rank, world, dev, dist)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, results, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, None, traceback.format_exc()))


def _ddp_gpt(rank, world, dev, dist):
    """DDP GPT-tiny over a "flexar" process group (a second group next to the gloo bootstrap) against one
    model trained on the whole batch in this process: max parameter difference after 4 SGD steps (the
    mean of the ranks' half-batch gradients vs the full-batch gradient: fp32 association only)."""
    import torch.nn as nn
    from torch.nn.parallel import DistributedDataParallel as DDP

    from allreduce_over_mpi_amd.models.gpt import GPT, PRESETS
    from allreduce_over_mpi_amd.parallel import backend  # noqa: F401 - registers "flexar"

    pg = dist.new_group(backend="flexar")
    torch.manual_seed(0)
    ref = GPT(PRESETS["gpt-tiny"]).to(dev)
    model = GPT(PRESETS["gpt-tiny"]).to(dev)
    model.load_state_dict(ref.state_dict())
    ddp = DDP(model, device_ids=[dev.index], process_group=pg, bucket_cap_mb=1)
    opt = torch.optim.SGD(ddp.parameters(), lr=0.05)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.05)
    g = torch.Generator().manual_seed(42)

    def loss(m, x, y):
        out = m(x)
        return nn.functional.cross_entropy(out.reshape(-1, out.shape[-1]), y.reshape(-1))

    for _ in range(4):
        t = torch.randint(0, 512, (2 * world, 65), generator=g).to(dev)
        x, y = t[:, :-1], t[:, 1:]
        sl = slice(2 * rank, 2 * rank + 2)
        opt.zero_grad()
        loss(ddp, x[sl], y[sl]).backward()
        opt.step()
        ropt.zero_grad()
        loss(ref, x, y).backward()
        ropt.step()
    torch.cuda.synchronize()
    diff = max((p - q).abs().max().item() for p, q in zip(model.parameters(), ref.parameters()))
    stats = getattr(pg, "stats", None)
    if stats is not None and stats.get("flexar_allreduce", 0) == 0:
        return float("inf")  # the flexar path must have carried the gradients
    return diff


def _run(world, shared, transport="rccl", no_ipc=False, parts=("all",), timeout=900):
    import queue

    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shared, q, transport, no_ipc, parts))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=timeout)
            assert err is None, f"rank {rank} failed:\n{err}"
            out[rank] = res
    except queue.Empty:
        pytest.fail(f"a rank did not finish within {timeout} s")
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return out


def _check(out, world, shared):
    for rank, res in out.items():
        topo, failed = res.pop("readiness")
        # connect-time probe and agreement; the self-test verified every protocol family on these links
        assert failed == [], (rank, failed, topo)
        assert topo["links_agreed"], topo
        if topo["ipc"]:
            assert topo["selftested"] == "fence,wt,ll,dma,rccl", topo
        for p in topo["peers"]:
            if p["rank"] != rank:
                assert p["link"] in (("same-device",) if shared else ("xgmi", "pcie")), topo
        if not shared and all(p["link"] == "xgmi" and p["hops"] <= 1 for p in topo["peers"] if p["rank"] != rank):
            assert topo["links"] == world - 1, topo
        for key, err in res.items():
            if key[0] == "fp8_emulation_mismatch":
                assert err < 2e-3, (rank, key, err)
                continue
            if key[0] == "fp8_rel":
                assert err < 0.1, (rank, key, err)
                continue
            if key[0] == "mx_mismatch":
                assert err == 0, (rank, key, err)
                continue
            if key[0] == "ddp":
                assert err < 2e-4, (rank, key, err)
                continue
            bf16 = any("bfloat16" in str(k) for k in key)
            # bf16: per-hop rounding may round h times - an explicit "+rw", or a multi-hop spec under the default
            # partials policy ("auto" takes "+rw" where it rounds <= 3 times); fp32 partials and flat round once
            spec = str(key[1]) if len(key) > 1 else ""
            single = "+f32" in spec or spec.split("+")[0] in ("flat", "oneshot", "ll", "dma") or spec.startswith("tree:%d" % world)
            tol = (1e-2 if single else 2e-2) if bf16 else 1e-5
            assert err < tol, (rank, key, err)


def _matrix_params():
    n = _ngpu()
    out = []
    for world in (2, 4, 8):
        if n >= world:
            out.append(pytest.param(world, False, id=f"n{world}-per-gpu"))
        elif world <= 4:
            out.append(pytest.param(world, True, id=f"n{world}-shared-gpu0"))
    return out


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world,shared", _matrix_params())
def test_acceptance_matrix(cuda, world, shared):
    _check(_run(world, shared), world, shared)


@pytest.mark.timeout(900)
@pytest.mark.skipif(_ngpu() >= 8, reason="the per-GPU n8 case of test_acceptance_matrix runs the whole matrix")
def test_acceptance_matrix_n8_shared(cuda):
    """The whole matrix at N = 8 with 8 ranks on device 0 - the schedules the driver's 8-GPU bench will time
    (full-mesh ring:7 from the Hamiltonian decomposition, mixed-radix trees 2,4 / 4,2 with push and pull,
    RHD, typed partials, fp8, zero copy, the other collectives, DDP) - so a planner or protocol bug at N = 8
    shows up before the first 8-GPU run."""
    _check(_run(8, True), 8, True)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("shared", [pytest.param(_ngpu() < 2, id="auto-device-map")])
def test_rccl_fallback_when_ipc_is_unavailable(cuda, shared):
    """Every peer mapping fails (FLEXAR_FAULT_NO_IPC): the communicator still comes up and every schedule
    (FlexTree, ring, RHD, flat) runs over the RCCL message transport with the same results."""
    world = 4 if _ngpu() >= 4 or shared else 2
    out = _run(world, shared, transport="auto", no_ipc=True, parts=("allreduce",))
    for rank, res in out.items():
        topo, failed = res.pop("readiness")
        assert topo["ipc"] is False and topo["rccl"] is True, topo
        assert topo["selftested"] == "rccl" and "rccl" not in failed, (topo, failed)
        for key, err in res.items():
            tol = 1e-5 if "float32" in str(key) else 1e-2
            assert err < tol, (rank, key, err)
