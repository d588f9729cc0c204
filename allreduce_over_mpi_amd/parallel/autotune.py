"""Online algorithm selection: measure the candidate schedules on THIS node and install the winners.

The reference chooses its tree offline: a closed-form cost model (cost_model/CostModel.h:82-120) prints a
structure and a human exports FT_TOPO. flexar's runtime selector starts from an xGMI alpha-beta-gamma model
(csrc/include/flexar/cost_model.hpp) and can be overridden by a measured table (FLEXAR_TUNE_FILE, written
offline by tools/flexar_tune.py). ``autotune`` does the measurement in-process, at start-up, on the
actual communicator:

    comm = Communicator()
    table = autotune(comm)          # collective: every rank calls it with the same arguments
    # comm.all_reduce(...) now uses the measured winner for each size class

For every size (x4 steps) each candidate is checked against ``torch.distributed.all_reduce`` of the
communicator's group on three consecutive calls with inputs x, x/2, x/4 (a stale staging line from either
of the two previous calls would change the result), then timed; the slowest rank's time counts. A
candidate that fails or times out on any rank is dropped; every rank has synchronised by then, so the
recorded timeout is cleared (epochs advance once per call on every rank, aborted or not) and the
measurement goes on with the same communicator.
"""
from __future__ import annotations

import math
import time
from typing import Optional, Sequence

from .. import _native as nv


def default_candidates(world: int, nbytes: int, esize: int = 4) -> list[str]:
    """The schedules worth measuring for ``nbytes`` on ``world`` ranks (bench.py, tools/flexar_tune.py and
    ``autotune`` share this list): latency protocols for small buffers, every flat-stage protocol, rings
    on 1, 2 and 4 arc-disjoint channels and on N - 1 (the full mesh: ``ring:7`` at N = 8), RHD, the
    two-stage FlexTree factorizations (each also on N - 1 link-balanced channels: ``rhd:7``, ``tree:4,2:7``)
    and the copy engines. The direction-balanced flat ("+bidir") joins the
    flat protocols: on xGMI its reduce-scatter reads and its all-gather writes share the links' two
    directions. For 16/8-bit elements (``esize`` < 4) every multi-hop schedule is measured twice: with fp32
    partials (the default typed staging, one rounding) and rounded per hop ("+rw", 16-bit partials on the
    links, up to +43 % fewer link bytes for a ring at N = 8)."""
    c = ["ll", "oneshot", "oneshot+wt"] if nbytes <= (1 << 20) else (["oneshot"] if nbytes <= (8 << 20) else [])
    c += ["flat+pull", "flat+push", "flat+pull+nts", "flat+push+nts", "flat+pull+wt", "flat+push+wt"]
    c += ["flat+bidir", "flat+bidir+nts", "flat+bidir+wt"]  # both link directions in one XFER
    maxc = len([d for d in range(1, world) if math.gcd(d, world) == 1])
    c += ["ring", "ring+wt"] + [f"ring:{k}{m}" for k in (2, 4) if k <= maxc for m in ("", "+wt")]
    try:  # every outgoing link: N - 1 arc-disjoint rings where the full decomposition exists (ring:7 at N = 8)
        full = nv.ring_order(world, 0, 1)[1]
    except Exception:  # noqa: BLE001 - no native library: the circulant rings only
        full = maxc
    if full > 4:
        c.append(f"ring:{full}")
    if world > 2 and (world & (world - 1)) == 0:
        c.append("rhd+pull")
        if world >= 4:  # N - 1 link-balanced channels: every stage on every link (planner.hpp build_tree_channels)
            c.append(f"rhd:{world - 1}+pull")
    if world >= 8 and world % 4 == 0:
        c += [f"tree:4,{world // 4}+pull", f"tree:{world // 4},4+pull"]
        if world <= 16:
            c += [f"tree:4,{world // 4}:{world - 1}+pull", f"tree:{world // 4},4:{world - 1}+pull"]
    if nbytes >= (1 << 20):
        c.append("dma")
    if esize < 4:  # the single-rounding trade-off, measured: per-hop rounded forms of the multi-hop schedules
        c += [s.replace("+wt", "") + "+rw" + ("+wt" if "+wt" in s else "") for s in c
              if (s.startswith("ring") or s.startswith("rhd") or (s.startswith("tree:") and "," in s))]
    return c


def autotune(comm, sizes: Optional[Sequence[int]] = None, dtype=None, candidates=None, iters: int = 0,
             install: bool = True, verbose: bool = False, calibrate: bool = True,
             rows_out: Optional[list] = None) -> list[tuple[int, str, float]]:
    """Measure and (``install``) apply a per-size algorithm table. Returns [(bytes, spec, busbw_GBps)].
    ``sizes``: buffer bytes (default 4 KiB .. 256 MiB, x4). Collective over the communicator's group.
    ``calibrate``: also fit the cost model to every measurement (``Communicator.calibrate``), so sizes
    between and beyond the measured ones are priced with this node's constants; ``rows_out`` collects the
    (spec, bytes, us) rows (max over ranks)."""
    import torch
    import torch.distributed as dist

    from ..utils.perf import busbw_gbps

    world = comm.world_size
    if world < 2:
        return []
    dtype = dtype or torch.float32
    es = torch.tensor([], dtype=dtype).element_size()
    sizes = list(sizes) if sizes else [4096 << (2 * k) for k in range(9)]
    dev = torch.device("cuda", comm.device)
    group = comm.group
    host_ref = dist.get_backend(group) == "gloo"

    def agree_max(*v: float) -> list:
        t = torch.tensor(list(v), dtype=torch.float64, device="cpu" if host_ref else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        return [float(a) for a in t.tolist()]

    table, rows = [], []
    tol = {torch.float32: 1e-5, torch.bfloat16: 2e-2, torch.float16: 4e-3}.get(dtype, 1e-5) * 4 * math.sqrt(world)
    for nbytes in sizes:
        n = max(1, nbytes // es)
        x = torch.randn(n, device=dev).to(dtype)
        y = torch.empty_like(x)
        ref = x.float().cpu() if host_ref else x.float()
        dist.all_reduce(ref, group=group)
        ref = ref.to(dev)
        scale = float(ref.abs().max().item()) + 1e-6
        reps = iters or max(3, min(100, int(2e8 // max(nbytes, 1))))
        best, best_t = None, float("inf")
        for spec in (candidates or default_candidates(world, n * es)):
            # exactly two agreements per candidate on every rank, whatever raised where: a rank that failed
            # its checks must not skip a collective its peers make (they would pair with its next one)
            failed, t = 0.0, 0.0
            try:
                for sc in (1.0, 0.5, 0.25):
                    xs = x if sc == 1.0 else (x.float() * sc).to(dtype)
                    comm.all_reduce(xs, out=y, algo=spec)
                    torch.cuda.synchronize()
                    if float((y.float() - ref * sc).abs().max().item()) > tol * scale * sc:
                        failed = 1.0
                comm.check()
            except nv.FlexarError:
                failed = 1.0
            failed, = agree_max(failed)
            if failed == 0.0:
                try:
                    torch.cuda.synchronize()
                    dist.barrier(group=group)
                    t0 = time.perf_counter()
                    for _ in range(reps):
                        comm.all_reduce(x, out=y, algo=spec)
                    torch.cuda.synchronize()
                    t = (time.perf_counter() - t0) / reps
                    comm.check()
                except nv.FlexarError:
                    failed = 1.0
            t, failed = agree_max(t, failed)
            if failed != 0.0:
                torch.cuda.synchronize()
                comm.clear_error()  # every rank is here, nothing in flight: a timeout must not poison the rest
                if verbose and comm.rank == 0:
                    print(f"[autotune] {n * es:>11d} B  {spec:16s} excluded (wrong or failed on a rank)", flush=True)
                continue
            rows.append({"spec": spec, "bytes": n * es, "us": t * 1e6})
            if verbose and comm.rank == 0:
                print(f"[autotune] {n * es:>11d} B  {spec:16s} {t * 1e6:10.2f} us  "
                      f"busbw {busbw_gbps(n * es, t, world):8.1f} GB/s", flush=True)
            if t < best_t:
                best, best_t = spec, t
        if best is not None:
            table.append((n * es, best, round(busbw_gbps(n * es, best_t, world), 2)))
        del x, y, ref
    if install and table:
        lines, prev = [], None
        for nbytes, spec, _ in table:
            if spec != prev:  # a row covers every size up to the next row
                lines.append(f"{world} {nbytes} {spec}")
                prev = spec
        comm.set_tune_table("\n".join(lines))
    if calibrate and install and hasattr(comm, "calibrate"):
        try:
            fit = comm.calibrate(rows)  # identical rows on every rank (max over ranks): identical model
            if verbose and comm.rank == 0:
                print(f"[autotune] cost model fitted: FLEXAR_MODEL={fit['FLEXAR_MODEL']} "
                      f"(median rel err {fit['median_rel_err']:.2f})", flush=True)
        except ValueError:
            pass  # too few executor measurements to fit 4 parameters
    if rows_out is not None:
        rows_out.extend(rows)
    return table
