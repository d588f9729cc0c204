#!/usr/bin/env python3
"""Flagship benchmark: allreduce bus bandwidth on N MI355X GPUs (one rank per GPU).

Metric and config are BASELINE.json's: "allreduce bus bandwidth (GB/s) vs buffer bytes, fp32/bf16, at
1/2/4/8 MI355X", headline buffer = config #2 (fp32, 256 MiB). The reference's own driver
(allreduce_over_mpi/benchmark.cpp:147-215) times MPI_Allreduce_FT with MPI_Barrier + MPI_Wtime on rank 0
only; here every rank is timed over K steps bracketed by barrier + device synchronize on both sides and
the MAX over ranks is reported.

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \\
        --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8

Numbers (rccl-tests convention): algbw = bytes / t and busbw = algbw * 2 (N - 1) / N. `value` IS the
busbw of BASELINE.json's metric, the figure rccl-tests prints (one number for the job: every rank moves
the same bytes), so `value == busbw_GBps` for every N and the 1/2/4/8 series is one quantity;
`vs_baseline` compares it with the reference's busbw. At N = 1 the busbw factor 2(N-1)/N is 0 (no
inter-GPU traffic), so `value` is 0 there by definition; the device-copy algbw of that run is reported
separately as `algbw_GBps` and is not comparable with busbw. `aggregate_busbw_GBps` (busbw x N) is kept
as an extra key for whole-job accounting.

At N >= 2 the same JSON line also measures every other BASELINE config, OUTSIDE the headline's timed
region, each next to RCCL and timed max-over-ranks:
  config3  bf16 1 GiB: RHD with fp32 partials ("+f32"), RHD rounded per hop ("+rw") and the selector's own
           choice, each checked against an fp32 reference, next to RCCL bf16;
  config4  the 4 KiB -> 1 GiB (x4) sweep of the selector's choice, every size an exact-integer correctness
           check, next to RCCL;
  config5  the fused-scale fp8 gradient allreduce (fp32 256 MiB in, OCP e4m3 on the links, AVG; amax pass +
           one executor launch) with its max relative error, next to RCCL fp32 AVG;
plus the cost model's own choice at the headline size (the connect-time calibrated selector, what `auto`
runs in production), the connect-time readiness result and calibration, and the start-up tuner's table.

Wall-clock budget: FLEXAR_BENCH_BUDGET_S (default 400 s, the driver allows 600). Optional items are
dropped in a fixed order when the budget runs short - first the calibration mini-sweep
(`cost_model_fit`), then config #4's tail sizes (>= 64 MiB), then the tuner's grid sweep - and every
dropped item is listed under `dropped`; `bench_wall_s` is the max over ranks of the time since start.
Skipping decisions use the max-over-ranks elapsed time, so every rank takes the same path.

Correctness: every tuner candidate and the final choice are checked against RCCL's result
(torch.distributed "nccl") on three consecutive calls whose inputs are scaled by 1, 1/2 and 1/4 (exact
in every dtype). Calls alternate staging halves, so a read of a staging line left over from one of the
two previous calls changes the result and is caught. The check runs again after the timed region.
Every failure is agreed on by all ranks (one max-over-ranks per candidate, whether or not this rank
raised), so ranks never diverge in their collective calls.
Data: synthetic torch.randn buffers seeded per rank. If no flexar algorithm is correct on this node the
run falls back to RCCL and says so in `config.algorithm` and `fallback`.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

_T_START = time.monotonic()
REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# the reference (FlexTree ring, FT_TOPO=1) at N=2, 256 MiB fp32 = 3.15 GB/s busbw per rank
# (measured locally on CPU/MPICH — the reference publishes no numbers).
BASELINE_BUSBW_256MIB = 3.15
CHECK_SCALES = (1.0, 0.5, 0.25)  # powers of two: exact scaling of inputs and of the reference sum
CALIB_SIZES = (64 << 10, 1 << 20, 8 << 20, 64 << 20)
# budget fractions: an optional item runs only if the agreed elapsed time is below this share of the budget.
# A lower share = dropped sooner as the run eats its budget: the calibration mini-sweep first, then config
# #4's tail sizes, then the grid sweep (priority order; the grid sweep, checked right after the tuner, goes
# only when the tuner alone has spent three quarters of the budget)
DROP_AT = {"cost_model_fit": 0.5, "config4_tail": 0.65, "grid_sweep": 0.75}
COMPANION_AT = 0.85  # config3 / config4 head / config5 / small messages


def write_line(fd: int, text: str):
    """One whole line with ONE write(2) where the OS allows (a pipe takes up to PIPE_BUF = 4 KiB atomically): every
    rank of a torchrun job shares the launcher's stdout / stderr, and print() issues the text and its newline as two
    writes, so another rank's line could land between them - or inside rank 0's JSON line."""
    (sys.stdout if fd == 1 else sys.stderr).flush()
    data = (text + "\n").encode()
    while data:
        n = os.write(fd, data)
        data = data[n:]


def log(rank, *a):
    if rank == 0:
        write_line(2, " ".join(["[bench]"] + [str(x) for x in a]))


_NV = None  # the native module once imported (phase breadcrumbs)


def phase(rank, what):
    """A phase line from EVERY rank (a fault on rank k names the phase rank k reached):
    rank, wall-clock time (comparable with torch's / RCCL's log stamps) and seconds since this process
    started, on stderr; also a native breadcrumb that the crash report prints."""
    now = time.time()
    stamp = time.strftime("%H:%M:%S", time.localtime(now)) + f".{int(now * 1000) % 1000:03d}"
    write_line(2, f"[phase r{rank} {stamp} +{time.monotonic() - _T_START:.3f}s] bench: {what}")
    if _NV is not None:
        _NV.crumb("phase", "bench: " + what, rank)


class RcclOnly:
    """Stand-in communicator when flexar cannot run on this node: every call is RCCL's allreduce."""

    def __init__(self, dist):
        self.dist = dist
        self.calibration = None

    def all_reduce(self, tensor, op="sum", out=None, algo=None, scale=1.0):
        dst = tensor if out is None else out.copy_(tensor)
        self.dist.all_reduce(dst, op=self.dist.ReduceOp.AVG if op == "avg" else self.dist.ReduceOp.SUM)
        return dst

    def check(self):
        pass

    def set_grid(self, g):
        pass

    def describe(self, count, dtype):
        return "rccl"

    def close(self):
        pass


class Budget:
    """Wall-clock budget of the whole run; decisions on the max-over-ranks elapsed time (collective)."""

    def __init__(self, seconds, agree):
        self.seconds = seconds
        self.agree = agree
        self.dropped = []

    def elapsed(self):
        return self.agree(time.monotonic() - _T_START)

    def allow(self, item, fraction):
        """Collective: True if the agreed elapsed time leaves room for `item` (else it is listed as dropped)."""
        e = self.elapsed()
        if e <= fraction * self.seconds:
            return True
        self.dropped.append({"item": item, "elapsed_s": round(e, 1), "limit_s": round(fraction * self.seconds, 1)})
        return False


def configure_env(world: int, rank: int, local: int, environ) -> tuple:
    """The environment of one bench rank, set before HIP initialises; returns (local device, shared,
    shared_rccl). One GPU per rank (the driver's N-GPU run) gets nothing shared-GPU-specific: no hardware
    queue cap and no grid clamp (tests/test_bench_launch.py pins this).

    FLEXAR_BENCH_SHARED_GPU=1: rehearsal of the multi-rank flow with every rank on device 0 (a 1-GPU box).
    By default the reference result and barriers use gloo and the RCCL comparison is skipped; the numbers
    measure one shared HBM, not xGMI. FLEXAR_BENCH_SHARED_RCCL=1 (with SHARED_GPU): the driver's own flow on
    one GPU - "nccl" process group, RCCL reference and comparator, the '+rccl' message-transport candidates.
    RCCL refuses two ranks on one GPU of one host, so every rank gets its own NCCL_HOSTID: RCCL then treats
    the ranks as separate hosts and carries their messages over its socket transport on loopback (RCCL
    numbers are not xGMI figures)."""
    shared = environ.get("FLEXAR_BENCH_SHARED_GPU", "0") == "1"
    shared_rccl = shared and world > 1 and environ.get("FLEXAR_BENCH_SHARED_RCCL", "0") == "1"
    if shared_rccl:
        environ["NCCL_HOSTID"] = f"flexar-bench-rank{rank}"  # must differ per rank
        environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        environ.setdefault("NCCL_IB_DISABLE", "1")
    if shared:
        local = 0
        # 8 processes x HIP's default 4 hardware queues oversubscribe the GPU's compute queues: the command
        # processor then time-slices the processes and every cross-rank hand-off waits for a queue switch
        # (measured: 28.6 ms instead of 1.0 ms per 256 MiB call at N = 8). Set before HIP initialises. A cap,
        # not a default: the GPU box exports HIP's own default (4) explicitly (profiles/r4_rehearsal).
        if world > 4 and int(environ.get("GPU_MAX_HW_QUEUES", "4") or 4) > 2:
            environ["GPU_MAX_HW_QUEUES"] = "2"
        # every rank's workgroups must be co-resident on the one GPU (they spin on each other)
        environ.setdefault("FLEXAR_MAX_GRID", str(max(8, 256 // (2 * world))))
    return local, shared, shared_rccl


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n: int, child_argv, python=None, timeout_s=None) -> int:
    """`bench.py --gpus N` with no launcher (WORLD_SIZE unset): start the N ranks here, one process per GPU,
    like the reference's driver is started by mpiexec and reads MPI_Comm_size (allreduce_over_mpi/
    benchmark.cpp:48-52). This process makes NO GPU call (HIP is initialised only in the children, which
    are started as new processes, never exec'd over this one); each child gets RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT, rank 0's stdout (the JSON line) is passed through, every other
    rank's stdout goes to stderr. A failed rank ends the others; the exit code is the first failure's."""
    import subprocess
    import threading

    port = _free_port()
    procs, lines = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([python or sys.executable] + list(child_argv), env=env,
                                      stdout=subprocess.PIPE, text=True))

    def pump(r):  # every rank's stdout, line by line (a full pipe must never stall a rank)
        for line in procs[r].stdout:
            if r == 0 and line.lstrip().startswith("{"):
                lines.append(line)
            else:
                sys.stderr.write(line)

    pumps = [threading.Thread(target=pump, args=(r,), daemon=True) for r in range(n)]
    for t in pumps:
        t.start()
    t0 = time.monotonic()
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        failed = [c for c in codes if c not in (None, 0)]
        if failed and not rc:
            rc = failed[0]
            print(f"[bench] a rank exited with {rc}: stopping the others", file=sys.stderr, flush=True)
            for p in procs:
                if p.poll() is None:
                    p.terminate()
        if all(c is not None for c in codes):
            break
        if timeout_s and time.monotonic() - t0 > timeout_s:
            for p in procs:
                if p.poll() is None:
                    p.kill()
            rc = rc or 124
        time.sleep(0.05)
    for t in pumps:
        t.join(timeout=10)
    js = lines
    if js and rc == 0:
        print(js[-1].rstrip("\n"), flush=True)
    elif rc == 0:
        print("[bench] rank 0 printed no JSON line", file=sys.stderr, flush=True)
        rc = 1
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size-mb", type=float, default=256.0, help="buffer MiB per rank")
    ap.add_argument("--dtype", default="float32", choices=["float32", "bfloat16", "float16", "float8_e4m3fn"])
    ap.add_argument("--op", default="sum", choices=["sum", "avg"],
                    help="avg = sum with the 1/N post-scale fused into the reduction (fp8 gradients)")
    ap.add_argument("--sweep", default="", help="MIN:MAX bytes (e.g. 4K:4G): busbw table vs RCCL, x4 steps")
    ap.add_argument("--sweep-out", default="", help="write sweep rows as JSON lines here (rank 0)")
    ap.add_argument("--tune-out", default="", help="append the tuner's choice as a FLEXAR_TUNE_FILE line")
    ap.add_argument("--algo", default="auto", help="flexar algorithm spec or 'auto' (tuned at start-up)")
    ap.add_argument("--no-rccl", action="store_true", help="skip the RCCL comparison run")
    ap.add_argument("--no-small", action="store_true", help="skip the 8 KiB latency companion figure")
    ap.add_argument("--no-tune", action="store_true", help="use the cost model instead of the start-up tuner")
    ap.add_argument("--no-calibrate", action="store_true",
                    help="skip the 64 KiB..64 MiB mini-sweep of the tuner's candidates vs RCCL and the cost-model fit")
    ap.add_argument("--no-configs", action="store_true", help="skip the BASELINE config #3/#4/#5 companion sections")
    ap.add_argument("--config3-mb", type=float, default=1024.0, help="config #3 buffer MiB (bf16)")
    ap.add_argument("--config4-max", default="4G", help="config #4 sweep top size (BASELINE: 4 KB -> 4 GB)")
    ap.add_argument("--config5-mb", type=float, default=256.0, help="config #5 buffer MiB (fp32 in, e4m3 wire)")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "auto", "ipc"],
                    help="Communicator transport at N > 1 (rccl: IPC + the '+rccl' message transport candidates)")
    ap.add_argument("--no-reduce-kernel", action="store_true",
                    help="N = 1: skip the fan-in 2/4/8 reduction-kernel section (reduce_kernel)")
    ap.add_argument("--reduce-kernel-mb", type=float, default=256.0, help="reduce_kernel: MiB per source")
    ap.add_argument("--no-group-executor", action="store_true",
                    help="N = 1: skip the 8-ranks-in-one-launch executor section (group_executor)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: this process starts the N ranks itself (and never touches the GPU)
        sys.exit(self_launch(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # every rank's Python stacks on stderr if the run is still going after this long (a stuck collective
    # then names itself in the log); FLEXAR_BENCH_TRACEBACK_S=0 disables it
    tb_s = int(os.environ.get("FLEXAR_BENCH_TRACEBACK_S", "540" if world > 1 else "0"))
    if tb_s > 0:
        import faulthandler

        faulthandler.dump_traceback_later(tb_s, repeat=True)
    if world > 1:  # every rank's start-up phases on stderr (the Python communicator's too)
        os.environ.setdefault("FLEXAR_PHASE_LOG", "1")
    phase_log = os.environ.get("FLEXAR_PHASE_LOG") == "1"
    ph = (lambda what: phase(rank, what)) if phase_log else (lambda what: None)
    ph(f"start (world {world}, local rank {local})")

    import torch
    import torch.distributed as dist

    ph("torch imported")
    local, shared, shared_rccl = configure_env(world, rank, local, os.environ)
    host_ref = shared and not shared_rccl  # gloo process group: references and reductions on the host
    if shared:
        args.no_rccl = args.no_rccl or not shared_rccl
    ndev = torch.cuda.device_count()
    if not shared and ndev and local >= ndev:
        # a launcher that restricts each rank to its own GPU (HIP_VISIBLE_DEVICES per rank): that GPU is device 0
        log(rank, f"LOCAL_RANK {local} but {ndev} visible device(s): using device {local % ndev}")
        local = local % ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ph(f"device {local} set")
    # the native library (and its fatal-signal / terminate report) before the process group: a fault inside
    # torch's eager RCCL initialisation - where the round-4 rehearsal fault surfaced, docs/ROUND5.md - then
    # prints this rank's breadcrumbs too, which show that no flexar launch had been issued
    from allreduce_over_mpi_amd import _native as nv

    global _NV
    nv.lib()
    _NV = nv
    nv._T0 = _T_START  # the communicator's phase lines count from this process's start too
    ph("native library loaded")
    if world > 1:
        if host_ref:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        ph("process group ready (" + ("gloo" if host_ref else "nccl, eager RCCL init") + ")")
    if args.gpus != world:
        log(rank, f"note: --gpus {args.gpus} but WORLD_SIZE={world}; benchmarking {world} rank(s)")

    from allreduce_over_mpi_amd.parallel.comm import Communicator
    from allreduce_over_mpi_amd.utils.perf import algbw_gbps, busbw_gbps

    dtype = getattr(torch, args.dtype)
    esize = torch.tensor([], dtype=dtype).element_size()
    nbytes = int(args.size_mb * (1 << 20))
    count = nbytes // esize
    nbytes = count * esize

    os.environ.setdefault("FLEXAR_TIMEOUT_MS", "5000")  # a broken candidate costs seconds, not minutes
    # staging for one whole call (flat pull: N landing blocks + N published blocks per parity half), so a
    # 256 MiB allreduce is ONE launch; 288 GB of HBM makes 1 GiB of workspace per rank free
    ws_bytes = max(512 << 20, 4 * nbytes + (64 << 20))
    fallback = None

    def max_over_ranks(v: float) -> float:
        if world == 1:
            return v
        t = torch.tensor([v], device="cpu" if host_ref else dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def max_vec(vals):
        if world == 1:
            return list(vals)
        t = torch.tensor(list(vals), device="cpu" if host_ref else dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [float(v) for v in t.tolist()]

    budget = Budget(float(os.environ.get("FLEXAR_BENCH_BUDGET_S", "400")), max_over_ranks)

    # one rank per GPU: IPC plus the RCCL message transport, so the tuner also measures the FlexTree / ring /
    # RHD schedules over ncclSend/ncclRecv ("+rccl"); if RCCL cannot be set up, IPC alone
    transports = ["ipc"] if (world == 1 or host_ref) else [args.transport, "ipc"] if args.transport != "ipc" else ["ipc"]

    creations = []  # one entry per communicator this run built (rebuilds included): what readiness did

    def make_comm():
        err = None
        for tr in transports:
            try:
                cm = Communicator(workspace_bytes=ws_bytes, transport=tr)
                creations.append(creation_record(cm, tr))
                return cm
            except nv.FlexarError as e:
                err = e
                if world > 1 and not shared:
                    log(rank, f"flexar communicator with transport={tr} failed: {e}")
        if world == 1 or shared:
            raise err
        log(rank, f"flexar communicator unavailable on this node ({err}); measuring RCCL instead")
        return None

    t_phase = time.perf_counter()
    ph("communicator creation")
    comm = make_comm()
    ph(f"communicator ready after {time.perf_counter() - t_phase:.1f} s")
    if comm is None:
        comm, fallback = RcclOnly(dist), "flexar communicator could not be created"
    # the three buffers first, each its own allocation (registration maps whole allocations into the peers;
    # a temporary freed first would leave a larger block the allocator carves them from)
    x = torch.empty(count, device=dev, dtype=dtype)
    y = torch.empty_like(x)
    xs = torch.empty_like(x)  # scaled copies of x for the stale-staging check
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    x0 = torch.randn(count, device=dev, dtype=torch.float32, generator=gen)
    if dtype == torch.float8_e4m3fn:
        x0 = x0 * 8  # fp8 e4m3 range: |x| <= 448
    x.copy_(x0.to(dtype))
    del x0
    zc_note = None

    def register_buffers(cm):
        """Register x, xs and y for the zero-copy candidates ("+zc": the flat schedule reads the peers'
        buffers over IPC, no staging). Collective; a failure on any rank drops the candidates everywhere."""
        nonlocal zc_note
        if world == 1 or not isinstance(cm, Communicator):
            return False
        if os.environ.get("FLEXAR_BENCH_ZC", "1") == "0":
            zc_note = "disabled (FLEXAR_BENCH_ZC=0)"
            return False
        try:
            cm.register_many([x, xs, y])
            return True
        except nv.FlexarError as e:
            zc_note = f"registration failed: {e}"
            log(rank, f"zero-copy candidates skipped: {e}")
            return False

    def rebuild(why):
        """Collective: a failed call may leave epochs / flags inconsistent - start from a fresh communicator.
        close() is collective in the library (flexar_comm_destroy agrees with every peer that all calls have
        finished and that every rank has unmapped before anything is freed), so the next communicator's
        memory is never allocated, exported or mapped while a peer still maps the old one."""
        nonlocal comm, fallback
        comm.close()
        comm = make_comm() or RcclOnly(dist)
        if isinstance(comm, RcclOnly):
            fallback = f"flexar communicator could not be rebuilt ({why})"

    zc = False  # registered after the cost-model measurement (which runs the unregistered, staging path)

    # ---------------------------------------------------------------- correctness vs RCCL
    op = args.op
    if dtype == torch.float8_e4m3fn and not host_ref:  # RCCL reference computed in fp32 from the same fp8 inputs
        ref = x.float()
        if world > 1:
            dist.all_reduce(ref)
        ref = (ref / world if op == "avg" else ref).to(dtype)
    elif host_ref:  # gloo: reference on the host
        ref = x.float().cpu()
        if world > 1:
            dist.all_reduce(ref)
        ref = (ref / world if op == "avg" else ref).to(dev).to(dtype)
    else:
        ref = x.clone()
        if world > 1:
            dist.all_reduce(ref, op=dist.ReduceOp.AVG if op == "avg" else dist.ReduceOp.SUM)
    ref_f = ref.float()
    ph(f"RCCL reference ready after {time.perf_counter() - t_phase:.1f} s")
    ref_max = float(ref_f.abs().max().item()) + 1e-6
    tol = {torch.float32: 1e-5, torch.bfloat16: 2e-2, torch.float16: 4e-3, torch.float8_e4m3fn: 0.13}[dtype]
    tol = tol * math.sqrt(world) * 4 if dtype != torch.float8_e4m3fn else tol

    def check(spec):
        """Local (no collectives): three consecutive calls with inputs x, x/2, x/4 - every result must match
        the reference scaled the same way (a stale staging line from either of the two previous calls would
        be off by 2x/4x). Returns (failed, err): failed 0 ok, 0.5 wrong result, 1 error (the communicator
        may be inconsistent); the caller agrees on it with every rank."""
        worst = 0.0
        try:
            for s in CHECK_SCALES:
                src = x
                if s != 1.0:
                    xs.copy_((x.float() * s).to(dtype))
                    src = xs
                comm.all_reduce(src, out=y, op=op, algo=None if spec == "auto" else spec)
                torch.cuda.synchronize()
                err = float((y.float() - ref_f * s).abs().max().item()) / (ref_max * s)
                worst = max(worst, err)
            comm.check()
        except nv.FlexarError as e:
            return 1.0, str(e)
        return (0.0 if worst <= tol else 0.5), worst

    def verify(out, n):
        """A prefix of n elements of the last result against the same prefix of the reference."""
        err = float((out.float() - ref_f[:n]).abs().max().item()) / ref_max
        return err <= tol, err

    def timed_fn(fn, iters, warm=1):
        """Collective: per-call seconds (max over ranks) of fn, or None if it failed on any rank. Exactly two
        agreements on every rank whether or not this rank raised: a warm-up failure anywhere skips the timed
        calls everywhere (the peers would otherwise wait out the device watchdog on every timed call), and
        that first agreement is also the barrier that starts the clock together."""
        failed = 0.0
        try:
            for _ in range(warm):
                fn()
            torch.cuda.synchronize()
        except nv.FlexarError:
            failed = 1.0
        if world > 1:
            failed, = max_vec([failed])
        t0 = time.perf_counter()
        try:
            if not failed:
                for _ in range(iters):
                    fn()
                torch.cuda.synchronize()
                comm.check()
        except nv.FlexarError:
            failed = 1.0
        dt, bad = max_vec([time.perf_counter() - t0, failed])
        return None if bad else dt / iters

    def timed(spec, iters, warm=1):
        a = None if spec == "auto" else spec
        return timed_fn(lambda: comm.all_reduce(x, out=y, op=op, algo=a), iters, warm)

    # ---------------------------------------------------------------- cost model (no tune table)
    model = None
    if world > 1 and not fallback:
        ph("cost-model measurement")
        choice = comm.describe(count, dtype)
        spec0 = choice.split(" ")[0]
        failed0, err0 = check("auto")
        failed0 = max_over_ranks(failed0)
        t0_model = timed("auto", 5) if failed0 == 0.0 else None
        model = {"choice": choice, "predicted_us": round(comm.predict_us(spec0, nbytes), 1),
                 "measured_us": round(t0_model * 1e6, 1) if t0_model else None,
                 "busbw_GBps": round(busbw_gbps(nbytes, t0_model, world), 2) if t0_model else None,
                 "correct": failed0 == 0.0, "error": err0 if isinstance(err0, str) else None}
        log(rank, f"cost model: {choice} predicted {model['predicted_us']} us, measured {model['measured_us']} us")
        if failed0 >= 1.0 or (failed0 == 0.0 and t0_model is None):
            rebuild("cost-model measurement failed")
    zc = register_buffers(comm)
    if model and model["correct"] and zc and not isinstance(comm, RcclOnly):
        # the same automatic choice once the buffers are registered: the flat schedule (or any choice the
        # model prices higher than the zero-copy push form) runs "+zc+push" (comm.hip, FLEXAR_ZC_AUTO)
        f1, _ = check("auto")
        f1 = max_over_ranks(f1)
        t1 = timed("auto", 5) if f1 == 0.0 else None
        model["registered_choice"] = comm.last_spec() if hasattr(comm, "last_spec") else None  # after the zc decision
        model["registered_measured_us"] = round(t1 * 1e6, 1) if t1 else None
        model["registered_busbw_GBps"] = round(busbw_gbps(nbytes, t1, world), 2) if t1 else None
        model["registered_correct"] = f1 == 0.0
        if f1 >= 1.0 or (f1 == 0.0 and t1 is None):
            rebuild("registered cost-model measurement failed")
            zc = register_buffers(comm)

    # ---------------------------------------------------------------- start-up tuner
    algo = args.algo
    tune_log = {}
    calib = None
    timings = {}
    ranked = []  # (spec, grid) in the order the timed region tries them
    if fallback:
        algo = "rccl"
    elif world > 1 and algo == "auto" and not args.no_tune:
        from allreduce_over_mpi_amd.parallel.autotune import default_candidates

        # flat-stage protocols, rings on 1..4 arc-disjoint channels, RHD, two-stage FlexTree factorizations,
        # the copy engines (and the latency protocols for small buffers)
        cands = default_candidates(world, nbytes, esize=esize)
        ph(f"tuner ({len(cands)} candidates + registered / RCCL ones)")
        if comm.topology().get("rccl"):  # the schedules over RCCL send/recv as well
            cands += ["flat+rccl", "ring+rccl"] + (["rhd+rccl"] if world > 2 and not world & (world - 1) else [])
        if zc:  # registered buffers: the flat schedule straight from / to the peers' x and y (put: remote writes only)
            cands += ["flat+zc", "flat+zc+nts", "flat+zc+wt", "flat+zc+push", "flat+zc+push+nts", "flat+zc+push+wt",
                      "flat+zc+put", "flat+zc+put+nts", "flat+zc+put+wt"]
        for spec in cands:
            ph(f"tuner candidate {spec}")
            failed, err = check(spec)
            failed = max_over_ranks(failed)  # one agreement per candidate, on every rank
            t = timed(spec, 5, warm=2) if failed == 0.0 else None
            if failed == 0.0 and t is None:
                failed = 1.0
            if failed:
                tune_log[spec] = f"WRONG (max rel err {err:.3g})" if failed < 1.0 and not isinstance(err, str) \
                    else f"error: {err}" if isinstance(err, str) else "failed on a peer"
                log(rank, f"tuner: {spec} excluded ({tune_log[spec]})")
                if failed >= 1.0:  # the communicator's epochs / flags may be inconsistent now
                    rebuild(f"tuner candidate {spec} failed")
                    if isinstance(comm, RcclOnly):
                        break
                    zc = register_buffers(comm)
                continue
            timings[spec] = t
            tune_log[spec] = round(busbw_gbps(nbytes, t, world), 2)
            log(rank, f"tuner: {spec:14s} {t*1e3:8.3f} ms  busbw {busbw_gbps(nbytes, t, world):8.1f} GB/s")
        if not timings or fallback:
            fallback = fallback or "no flexar algorithm produced correct results on this node"
            log(rank, f"tuner: {fallback}; measuring RCCL instead")
            algo = "rccl"
            if not isinstance(comm, RcclOnly):
                comm.close()
                comm = RcclOnly(dist)
        else:
            # workgroup count for the two fastest schedules (auto = one per 32 KiB, at most FLEXAR_MAX_GRID);
            # up to every workgroup the GPU keeps resident (occupancy x CUs, measured at comm creation): a
            # rank's workgroup b only ever waits for workgroup b of its peers, so one rank per GPU needs no
            # co-residency, but more resident workgroups keep more xGMI loads in flight. Ranks sharing one GPU
            # must stay co-resident with each other (FLEXAR_MAX_GRID caps them).
            ranked_specs = sorted(timings, key=timings.get)
            best, best_grid, best_t = ranked_specs[0], 0, timings[ranked_specs[0]]
            if budget.allow("grid_sweep", DROP_AT["grid_sweep"]):
                resident = int(comm.stats().get("resident_blocks") or 256)
                grids = [g for g in (32, 64, 128, 256, 512, 1024) if g <= resident and
                         (not shared or g <= int(os.environ["FLEXAR_MAX_GRID"]))]
                for spec in ranked_specs[:2]:
                    for g in grids:
                        comm.set_grid(g)
                        t = timed(spec, 5)
                        if t is None:  # failed on some rank: stop the sweep on a fresh communicator
                            tune_log[f"{spec}@grid{g}"] = "failed"
                            rebuild(f"grid sweep {spec}@{g} failed")
                            zc = register_buffers(comm)
                            break
                        tune_log[f"{spec}@grid{g}"] = round(busbw_gbps(nbytes, t, world), 2)
                        if t < best_t:
                            best, best_grid, best_t = spec, g, t
                    if isinstance(comm, RcclOnly):
                        break
            if not isinstance(comm, RcclOnly):
                comm.set_grid(best_grid)
            algo = best
            # the runners-up (auto grid) stand by in case the pick fails its final checks on this node
            ranked = [(best, best_grid)] + [(sp, 0) for sp in ranked_specs if sp != best][:2]
            log(rank, f"tuner: selected {algo} grid={best_grid or 'auto'}")
            if rank == 0 and args.tune_out:
                with open(args.tune_out, "a") as f:  # "nranks bytes spec" (cost_model.hpp TuneTable)
                    f.write(f"{world} {nbytes} {algo}\n")

    # ---------------------------------------------------------------- timed region
    # The chosen algorithm is checked right before and right after the timed steps (same protocol state). A
    # failure there - a protocol that passed the tuner's checks but not these, e.g. an intermittent visibility
    # problem on a node never seen before - must not lose the run: the next-fastest correct candidate takes
    # over (fresh communicator), then RCCL, and the JSON line names what was rejected and why.
    if not ranked:
        ranked = [(algo, None)]
    if world > 1 and not host_ref and algo != "rccl":
        ranked.append(("rccl", None))
    rejected = {}
    t_step = err = None
    desc = algo
    for attempt, (algo, grid) in enumerate(ranked):
        if algo == "rccl" and not isinstance(comm, RcclOnly):
            comm.close()
            torch.cuda.synchronize()
            comm = RcclOnly(dist)
        elif attempt > 0:  # the failed attempt may have left epochs / flags inconsistent
            comm.close()  # collective teardown (see rebuild)
            comm = make_comm() or RcclOnly(dist)
            if isinstance(comm, RcclOnly):
                rejected[algo] = "the flexar communicator could not be rebuilt"
                continue
            zc = register_buffers(comm)
            if "+zc" in algo and not zc:
                rejected[algo] = "zero-copy registration failed on the rebuilt communicator"
                continue
        if algo == "rccl":
            fallback = fallback or "every flexar candidate failed its final checks"
        if grid is not None:
            comm.set_grid(grid)
        failed, err = check(algo)
        if attempt == 0 and os.environ.get("FLEXAR_BENCH_REJECT_FIRST") == "1":  # rehearses this fallback chain
            failed, err = 1.0, "rejected by FLEXAR_BENCH_REJECT_FIRST=1"
        if max_over_ranks(failed) != 0.0:
            rejected[algo] = f"final check failed before timing ({err if isinstance(err, str) else f'max rel err {err:.3g}'})"
            log(rank, f"{algo}: {rejected[algo]}; trying the next candidate")
            continue
        desc = comm.describe(count, dtype) if algo == "auto" else algo
        ph(f"timed region: {algo} (attempt {attempt})")
        log(rank, f"correctness vs {'RCCL' if world > 1 else 'input'}: max rel err {err:.3g} (ok); running {desc}")
        a = None if algo == "auto" else algo
        run_failed = 0.0
        try:
            for _ in range(args.warmup):
                comm.all_reduce(x, out=y, op=op, algo=a)
            torch.cuda.synchronize()
        except nv.FlexarError:
            run_failed = 1.0
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        try:
            if not run_failed:
                for _ in range(args.steps):
                    comm.all_reduce(x, out=y, op=op, algo=a)
        except nv.FlexarError:
            run_failed = 1.0
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed, run_failed = max_vec([time.perf_counter() - t0, run_failed])
        t_step = elapsed / max(1, args.steps)
        # the timed calls must have produced correct results too (checked again right after, same protocol state)
        failed, err_after = check(algo) if not run_failed else (1.0, "a timed call failed")
        if max_over_ranks(failed) == 0.0:
            break
        rejected[algo] = f"failed after the timed run ({err_after})"
        log(rank, f"{algo}: {rejected[algo]}; trying the next candidate")
        t_step = None
    if t_step is None:
        raise SystemExit(f"no algorithm passed the final checks: {rejected}")
    if rejected and tune_log is not None:
        tune_log["rejected_after_tuning"] = rejected

    rccl_busbw = None
    if world > 1 and not args.no_rccl and dtype != torch.float8_e4m3fn:
        z = x.clone()
        rt = timed_fn(lambda: dist.all_reduce(z), max(1, args.steps), max(1, args.warmup))
        rccl_busbw = round(busbw_gbps(nbytes, rt, world), 2) if rt else None
        del z

    # ---------------------------------------------------------------- BASELINE configs #3 / #4 / #5
    ph("timed region done")
    sections = {}
    flex = not isinstance(comm, RcclOnly)
    if world > 1 and flex and not args.no_configs:
        ph("BASELINE configs #5 / #3 / #4")
        if budget.allow("config5", COMPANION_AT):
            sections["config5"] = run_config5(comm, world, dev, dist, timed_fn, max_vec, host_ref, args, rank)
        if budget.allow("config3", COMPANION_AT):
            sections["config3"] = run_config3(comm, world, rank, dev, dist, timed_fn, max_vec, host_ref, args)
        if budget.allow("config4", COMPANION_AT):
            tail_ok = budget.allow("config4_tail", DROP_AT["config4_tail"])
            hi = parse_bytes(args.config4_max)
            sections["config4"] = run_sweep(comm, world, rank, dev, torch.float32, "sum", dist, max_over_ranks,
                                            4096, hi if tail_ok else min(hi, 16 << 20), not args.no_rccl and not host_ref,
                                            timed_fn, args.sweep_out)
            if not tail_ok:
                sections["config4"]["dropped_sizes"] = [b for b in _x4(4096, hi) if b > (16 << 20)]

    # latency-bound companion figure (outside the timed region): an 8 KiB fp32 allreduce, eager, the
    # selector's choice (LL), against RCCL's on the same buffer
    small = None
    if world > 1 and not args.no_small and budget.allow("small_msg", COMPANION_AT):
        xsm = torch.randn(2048, device=dev)
        ysm = torch.empty_like(xsm)
        tf = timed_fn(lambda: comm.all_reduce(xsm, out=ysm), 200, 20)
        small = {"flexar": round(tf * 1e6, 2) if tf else None}
        if not args.no_rccl and not host_ref:
            tr = timed_fn(lambda: dist.all_reduce(xsm), 200, 20)
            small["rccl"] = round(tr * 1e6, 2) if tr else None

    # calibration mini-sweep of the tuner's candidates vs RCCL + the cost-model fit (the first item dropped)
    if timings and flex and not args.no_calibrate and world > 1 and \
            budget.allow("cost_model_fit", DROP_AT["cost_model_fit"]):
        calib = calibrate_model(comm, timings, nbytes, esize, world, x, y, op, dist, max_over_ranks, rank, shared,
                                verify, world > 1 and not args.no_rccl and dtype != torch.float8_e4m3fn)

    algbw = algbw_gbps(nbytes, t_step)
    busbw = busbw_gbps(nbytes, t_step, world)
    # this rank's HBM traffic per step over the step time: the timed schedule's bytes from the program-cost
    # model (which matches rocprofv3 FETCH/WRITE_SIZE within 2.2 %, profiles/r3_pmc_model); N = 1: the copy
    # and the peer traffic the same way: all bytes this rank's program moves over links (remote loads +
    # stores), and the busiest link's bytes summed over the phases (what bounds the schedule on xGMI)
    hbm_tbps = link_rate = None
    try:
        if world == 1:
            hbm_bytes = 2.0 * nbytes
        elif flex and algo != "rccl":
            pc = nv.program_cost(desc.split(" ")[0], rank, world, count, args.dtype)
            hbm_bytes = pc["hbm_read"] + pc["hbm_write"]
            link_rate = {"all_links_GBps": round(pc["link_bytes"] / t_step / 1e9, 2),
                         "busiest_link_GBps": round(pc["link_time_bytes"] / t_step / 1e9, 2)}
        else:
            hbm_bytes = None
        hbm_tbps = round(hbm_bytes / t_step / 1e12, 3) if hbm_bytes else None
    except Exception:  # noqa: BLE001 - a schedule the model does not price: the fields stay empty
        hbm_tbps = link_rate = None
    value = busbw  # rccl-tests busbw; 0 at N = 1 by definition (see the module docstring)
    readiness = None
    if world > 1 and isinstance(comm, Communicator):
        readiness = readiness_record(comm, creations)
    out = {
        "metric": "allreduce bus bandwidth (GB/s)",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_step * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(busbw / BASELINE_BUSBW_256MIB, 2) if (world > 1 and args.size_mb == 256.0) else None,
        "dtype": {"float32": "fp32", "bfloat16": "bf16", "float16": "fp16", "float8_e4m3fn": "fp8_e4m3"}[args.dtype],
        "data": "synthetic (torch.randn per rank, seeded); results checked against RCCL before and after timing"
                + ("; REHEARSAL: all ranks share one GPU ("
                   + ("RCCL over loopback sockets" if shared_rccl else "gloo reference")
                   + "), not an xGMI measurement" if shared else ""),
        "config": {
            "model": f"allreduce {args.dtype} {args.size_mb:g}MiB buffer per rank"
                     + (" (BASELINE config #2)" if args.dtype == "float32" and args.size_mb == 256 else ""),
            "op": op,
            "global_batch": nbytes,
            "seq_len": None,
            "parallelism": f"dp{world}",
            "algorithm": desc,
        },
        "value_definition": "busbw (rccl-tests: algbw * 2(N-1)/N); 0 at N=1 by definition",
        "busbw_GBps": round(busbw, 2),
        "algbw_GBps": round(algbw, 2),
        "aggregate_busbw_GBps": round(busbw * world, 2),
        "hbm_TBps_per_rank": hbm_tbps,  # HBM traffic of the timed schedule / step time (MI355X peak ~8 TB/s)
        "peer_traffic_per_rank": link_rate,  # program-cost link bytes / step time (N > 1)
        **rccl_fields(busbw, rccl_busbw, shared_rccl),
        "fallback": fallback,
        "tuner": tune_log or None,
        "cost_model": model,
        "cost_model_fit": calib,
        "readiness": readiness,
        "zero_copy": {"registered": zc, "note": zc_note} if world > 1 else None,
        "small_msg_8KiB_us_per_call": small,
    }
    out.update(sections)
    if args.sweep:
        lo, hi = (parse_bytes(t) for t in args.sweep.split(":"))
        out["sweep"] = run_sweep(comm, world, rank, dev, dtype, op, dist, max_over_ranks, lo, hi,
                                 world > 1 and dtype != torch.float8_e4m3fn and not args.no_rccl and not host_ref,
                                 timed_fn, args.sweep_out)
    if world == 1:
        out["note"] = ("N=1: no inter-GPU traffic, busbw = 0 by definition (value); algbw_GBps is the device copy "
                       "through the flexar executor kernel and is not comparable with busbw")
        if not args.no_reduce_kernel:  # outside the timed region; the headline `value` is unchanged
            out["reduce_kernel"] = run_reduce_kernel(dev, args.reduce_kernel_mb)
        if not args.no_group_executor:
            out["group_executor"] = run_group_executor(dev)
    out["dropped"] = budget.dropped or None
    out["budget_s"] = budget.seconds
    out["bench_wall_s"] = round(budget.elapsed(), 1)
    # the result line alone on the shared stdout: every rank's earlier output is out before it (barrier), no rank
    # writes while it goes out (barrier after), and it leaves in whole writes starting on a fresh line
    if world > 1:
        dist.barrier()
    if rank == 0:
        write_line(1, json.dumps(out))
    if world > 1:
        dist.barrier()
    ph("teardown")
    comm.close()
    if world > 1:
        dist.destroy_process_group()


def rccl_fields(busbw, rccl_busbw, shared_rccl):
    """The same-node bar: flexar's busbw over RCCL's on the same buffer, same ranks, same box
    (vs_baseline compares with the reference's CPU/MPICH number, which is context only). In the shared-GPU
    rehearsal RCCL runs over loopback sockets, so a ratio against it means nothing on xGMI:
    the figure moves to rccl_busbw_GBps_loopback and vs_rccl is null."""
    if shared_rccl:
        return {"rccl_busbw_GBps": None, "rccl_busbw_GBps_loopback": rccl_busbw, "vs_rccl": None}
    return {"rccl_busbw_GBps": rccl_busbw, "vs_rccl": round(busbw / rccl_busbw, 3) if rccl_busbw else None}


def _x4(lo, hi):
    out, b = [], lo
    while b <= hi:
        out.append(b)
        b *= 4
    return out


def _recover(comm):
    """After a failure every rank agreed on (so every rank has synchronised): forget the recorded watchdog
    timeout, so the next section's calls start clean instead of failing on the stale error (epochs advance
    once per call on every rank, aborted or not: DESIGN.md §12)."""
    try:
        import torch

        torch.cuda.synchronize()
        if hasattr(comm, "clear_error"):
            comm.clear_error()
    except Exception:  # noqa: BLE001 - best effort: the section already reports the failure
        pass


def run_config5(comm, world, dev, dist, timed_fn, max_vec, host_ref, args, rank):
    """BASELINE config #5: the fused-scale fp8 gradient allreduce. fp32 256 MiB per rank in and out, OCP
    e4m3 on the links, AVG: one amax pass + ONE executor launch whose first transfer quantises with the
    global pre-scale and whose last dequantises with the post-scale (Communicator.all_reduce_fp8). Max
    relative error against the exact fp32 AVG (RCCL's), and RCCL's own fp32 AVG time next to it."""
    import torch

    from allreduce_over_mpi_amd import _native as nv
    from allreduce_over_mpi_amd.utils.perf import busbw_gbps

    n = int(args.config5_mb * (1 << 20)) // 4
    g = torch.Generator(device=dev)
    g.manual_seed(777 + rank)
    x = torch.randn(n, device=dev, generator=g)
    y = torch.empty_like(x)
    ref = x.cpu() if host_ref else x.clone()
    dist.all_reduce(ref)
    ref = (ref / world).to(dev)
    out = {"what": f"all_reduce_fp8: fp32 {args.config5_mb:g} MiB per rank, e4m3 wire, AVG (amax + one fused launch)"}
    failed, err = 0.0, None
    try:
        comm.all_reduce_fp8(x, op="avg", out=y)
        torch.cuda.synchronize()
        err = float((y - ref).abs().max().item()) / (float(ref.abs().max().item()) + 1e-12)
    except nv.FlexarError as e:
        failed, err = 1.0, str(e)
    failed, = max_vec([failed])
    if failed:
        out["error"] = err if isinstance(err, str) else "failed on a peer"
        _recover(comm)
        return out
    t = timed_fn(lambda: comm.all_reduce_fp8(x, op="avg", out=y), 10, 2)
    if t is None:
        _recover(comm)
    errs = max_vec([err])
    out.update(flexar_us=round(t * 1e6, 1) if t else None,
               flexar_busbw_GBps=round(busbw_gbps(4 * n, t, world), 2) if t else None,
               max_rel_err=round(errs[0], 5),
               correct=errs[0] <= 0.13)  # e4m3: 3 mantissa bits, one rounding per contribution and result
    # the OCP MX form of the same wire: a scale per 32-element block inside the one launch, no amax pass
    failed, err = 0.0, None
    try:
        comm.all_reduce_fp8(x, op="avg", out=y, wire="mx_e4m3")
        torch.cuda.synchronize()
        err = float((y - ref).abs().max().item()) / (float(ref.abs().max().item()) + 1e-12)
    except nv.FlexarError as e:
        failed, err = 1.0, str(e)
    failed, = max_vec([failed])
    if failed:
        out["mx"] = {"error": err if isinstance(err, str) else "failed on a peer"}
        _recover(comm)
    else:
        tm = timed_fn(lambda: comm.all_reduce_fp8(x, op="avg", out=y, wire="mx_e4m3"), 10, 2)
        if tm is None:
            _recover(comm)
        errm = max_vec([err])
        out["mx"] = {"what": "wire mx_e4m3 (OCP MX, 32-element blocks, one launch)",
                     "flexar_us": round(tm * 1e6, 1) if tm else None,
                     "flexar_busbw_GBps": round(busbw_gbps(4 * n, tm, world), 2) if tm else None,
                     "max_rel_err": round(errm[0], 5), "correct": errm[0] <= 0.13}
    if not host_ref and not args.no_rccl:
        z = x.clone()
        tr = timed_fn(lambda: dist.all_reduce(z, op=dist.ReduceOp.AVG), 10, 2)
        out.update(rccl_fp32_avg_us=round(tr * 1e6, 1) if tr else None,
                   rccl_fp32_avg_busbw_GBps=round(busbw_gbps(4 * n, tr, world), 2) if tr else None)
    del x, y, ref
    return out


def creation_record(comm, transport):
    """What the readiness gate did while building one communicator (kept for every rebuild)."""
    return {"transport": transport, "retried": getattr(comm, "retried", None),
            "selftest_failed": list(getattr(comm, "selftest_failed", []) or []),
            "selftest_recovered": list(getattr(comm, "selftest_recovered", []) or []),
            "selftest_flaky": list(getattr(comm, "selftest_flaky", []) or [])}


def readiness_record(comm, creations=()):
    """The bench JSON's `readiness` block (a failure is never silent, as the reference's
    exit(1) in allreduce_over_mpi/mpi_mod.hpp:916 never is): the final communicator's probe (links, peer link
    classes), the families the self-test ran and disabled, the ones that failed once and passed on the
    second pass (`selftest_recovered`: kept, ranks share a GPU; `selftest_flaky`: disabled anyway, one GPU
    per rank), every rank's failure notes (truncated), whether creation was retried after an agreed failure,
    the transport note (IPC unavailable -> message transport), whether the host agreement page is joined and
    verified shared, the calibration, and the same facts for every communicator the run built."""
    topo = comm.topology()
    notes = {}
    for r, v in sorted((getattr(comm, "selftest_notes", None) or {}).items()):
        txt = " / ".join(v)
        notes[str(r)] = txt if len(txt) <= 300 else txt[:297] + "..."
    return {"links": topo["links"], "links_local": topo.get("links_local"), "selftested": topo["selftested"],
            "disabled": topo["disabled"],
            "peer_links": sorted({p["link"] for p in topo["peers"] if p["link"] != "self"}),
            "selftest_recovered": list(getattr(comm, "selftest_recovered", []) or []),
            "selftest_flaky": list(getattr(comm, "selftest_flaky", []) or []),
            "selftest_notes": notes or None,
            "retried": getattr(comm, "retried", None),
            "transport_note": getattr(comm, "transport_note", None),
            "host_page": {"joined": bool(topo.get("host_page")), "verified_shared": topo.get("host_page_shared"),
                          "note": getattr(comm, "host_page_note", None)},
            "calibration": getattr(comm, "calibration", None),
            "creations": list(creations) or None}


def run_group_executor(dev, ranks=8, mib=64, iters=5,
                       specs=("flat+pull", "rhd+pull", "rhd:7+pull", "tree:4,2:7+pull", "ring:7", "flat+zc+push")):
    """N = 1 companion section: the complete multi-rank device protocol (flags, epochs, both staging parities)
    with `ranks` ranks in ONE launch on this GPU (LocalGroup), fp32 `mib` MiB per rank, for the schedule
    families of the 8-GPU node - the link-balanced channelled trees among them (`rhd:7`, `tree:4,2:7`). Inputs are
    integers, so every partial sum is exact: `exact` compares every element of every rank's result with the
    sum. The "links" are this GPU's HBM, so the figure is the executor's effective HBM rate (program-cost bytes
    over time), not an xGMI bandwidth."""
    import torch

    from allreduce_over_mpi_amd import _native as nv
    from allreduce_over_mpi_amd.parallel import LocalGroup

    t0 = time.perf_counter()
    count = (mib << 20) // 4
    grp = LocalGroup(ranks, workspace_bytes=4 * (mib << 20))
    # the same workgroups per rank for every schedule: 28, a multiple of the 7 channels of rhd:7 / tree:4,2:7 /
    # ring:7 (a grid is rounded down to whole channels, which on its own would cost the channelled forms 1/8 of
    # their workgroups here: profiles/r6_channels/)
    grid = 28
    grp.set_grid(grid)
    rows = []
    try:
        pat = torch.remainder(torch.arange(count, device=dev, dtype=torch.int32), 251)
        xs = [(pat + r).float() for r in range(ranks)]
        want = (pat * ranks + ranks * (ranks - 1) // 2).float()
        del pat
        ys = [torch.empty_like(x) for x in xs]
        for spec in specs:
            row = {"spec": spec}
            try:
                for _ in range(2):  # both staging parities (the in-process "+zc" addresses the ranks' buffers directly)
                    grp.all_reduce(xs, "sum", outs=ys, algo=spec)
                torch.cuda.synchronize()
                row["exact"] = all(torch.equal(y, want) for y in ys)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(iters):
                    grp.all_reduce(xs, "sum", outs=ys, algo=spec)
                en.record()
                torch.cuda.synchronize()
                us = st.elapsed_time(en) * 1e3 / iters
                costs = [nv.program_cost(spec, r, ranks, count, "float32", links=1) for r in range(ranks)]
                hbm = sum(c["hbm_read"] + c["hbm_write"] for c in costs)
                row.update(us=round(us, 1), eff_hbm_TBps=round(hbm / (us * 1e-6) / 1e12, 3))
                grp.check()
            except nv.FlexarError as e:
                row["error"] = str(e)
            rows.append(row)
        del xs, ys, want
    finally:
        grp.close()
        torch.cuda.empty_cache()
    return {"what": f"{ranks} ranks x {mib} MiB fp32 in one launch on one GPU (LocalGroup, {grid} workgroups per "
                    "rank): the multi-rank protocol and schedules of the 8-GPU node, shared HBM instead of xGMI",
            "rows": rows,
            "wall_s": round(time.perf_counter() - t0, 2)}


def run_reduce_kernel(dev, mib=256.0, fanins=(2, 4, 8), dtypes=("float32", "bfloat16", "float8_e4m3fn"), iters=10):
    """N = 1 companion section: the hand-written gfx950 fan-in reduction kernel that is
    the reference's hot loop (reduce_sum, allreduce_over_mpi/mpi_mod.hpp:245-452), measured by the driver's
    own run. dst = src_0 + ... + src_{K-1} over `mib` MiB sources (flexar_reduce: 16-B loads, fp32
    accumulation, one rounding to the dtype); effective HBM rate = (K + 1) x bytes / time (K reads + one
    write). Checked against the order-defined fp32 sum in torch (((s0 + s1) + s2) + ...), rounded once to the
    dtype: `bit_exact` is an exact comparison of every element, `max_rel_err` the largest |out - ref| over
    max |ref| (fp32 accumulation, so exact in every dtype unless the kernel's rounding differs)."""
    import torch

    from allreduce_over_mpi_amd.ops import reduce as flexar_reduce

    rows = []
    t0 = time.perf_counter()
    gen = torch.Generator(device=dev)
    for dname in dtypes:
        dt = getattr(torch, dname)
        es = torch.tensor([], dtype=dt).element_size()
        n = int(mib * (1 << 20)) // es
        srcs = []
        for k in range(max(fanins)):
            gen.manual_seed(99 + k)
            srcs.append(torch.randn(n, device=dev, generator=gen).to(dt))
        out = torch.empty_like(srcs[0])
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for k in fanins:
            sk = srcs[:k]
            for _ in range(2):
                flexar_reduce(sk, "sum", out=out)
            torch.cuda.synchronize()
            st.record()
            for _ in range(iters):
                flexar_reduce(sk, "sum", out=out)
            en.record()
            torch.cuda.synchronize()
            t = st.elapsed_time(en) / iters * 1e-3
            ref = sk[0].float()
            for s in sk[1:]:
                ref = ref + s.float()
            ref_d = ref.to(dt)
            exact = bool(torch.equal(out.view(torch.uint8), ref_d.view(torch.uint8)))
            err = float((out.float() - ref).abs().max().item()) / (float(ref.abs().max().item()) + 1e-30)
            rows.append({"dtype": dname, "fanin": k, "bytes_per_src": n * es, "us": round(t * 1e6, 1),
                         "eff_TBps": round((k + 1) * n * es / t / 1e12, 3), "bit_exact": exact,
                         "max_rel_err": float(f"{err:.3g}")})
            del ref, ref_d
        del srcs, out
        torch.cuda.empty_cache()
    return {"what": "flexar_reduce: dst = sum of K sources (fp32 accumulate), effective TB/s = (K+1) x bytes / time; "
                    "checked against torch's order-defined fp32 sum rounded once to the dtype",
            "rows": rows, "wall_s": round(time.perf_counter() - t0, 2)}


def run_config3(comm, world, rank, dev, dist, timed_fn, max_vec, host_ref, args):
    """BASELINE config #3: bf16, 1 GiB per rank. RHD (tree 2,..,2) with fp32 partials ("+f32": one rounding)
    and rounded per hop ("+rw": the reference's ring semantics, bf16 partials on the links), single-channel and
    with N - 1 link-balanced channels ("rhd:7" at N = 8), and the
    selector's own choice, each checked against the fp32 sum of the same bf16 inputs, next to RCCL bf16."""
    import torch

    from allreduce_over_mpi_amd import _native as nv
    from allreduce_over_mpi_amd.utils.perf import busbw_gbps

    nbytes = int(args.config3_mb * (1 << 20))
    n = nbytes // 2
    g = torch.Generator(device=dev)
    g.manual_seed(4242 + rank)
    x = torch.randn(n, device=dev, generator=g).to(torch.bfloat16)
    y = torch.empty_like(x)
    ref = x.float().cpu() if host_ref else x.float()
    dist.all_reduce(ref)
    ref = ref.to(dev)
    ref_max = float(ref.abs().max().item()) + 1e-6
    out = {"what": f"bf16 {args.config3_mb:g} MiB per rank", "bytes": n * 2, "variants": {}}
    pow2 = world > 1 and not world & (world - 1)
    # single-channel RHD drives one xGMI link per stage; rhd:C (C = N - 1 link-balanced channels, planner.hpp
    # build_tree_channels) spreads every stage over all of them
    variants = (["rhd+pull+f32", "rhd+pull+rw"] if pow2 else []) + \
               ([f"rhd:{world - 1}+pull+f32", f"rhd:{world - 1}+pull+rw"] if pow2 and world >= 4 else []) + ["auto"]
    for spec in variants:
        a = None if spec == "auto" else spec
        failed, err = 0.0, None
        try:
            comm.all_reduce(x, out=y, algo=a)
            torch.cuda.synchronize()
            err = float((y.float() - ref).abs().max().item()) / ref_max
            comm.check()
        except nv.FlexarError as e:
            failed, err = 1.0, str(e)
        failed, = max_vec([failed])
        row = {"spec": comm.describe(n, torch.bfloat16).split(" ")[0] if spec == "auto" else spec}
        if failed:
            row["error"] = err if isinstance(err, str) else "failed on a peer"
            out["variants"][spec] = row
            _recover(comm)
            continue
        t = timed_fn(lambda: comm.all_reduce(x, out=y, algo=a), 5, 1)
        if t is None:
            _recover(comm)
        e = max_vec([err])[0]
        row.update(us=round(t * 1e6, 1) if t else None, busbw_GBps=round(busbw_gbps(n * 2, t, world), 2) if t else None,
                   max_rel_err=round(e, 6), correct=e <= 2e-2 * math.sqrt(world) * 4)
        out["variants"][spec] = row
        log(rank, f"config3 {spec}: {row}")
    if not host_ref and not args.no_rccl:
        z = x.clone()
        tr = timed_fn(lambda: dist.all_reduce(z), 5, 1)
        z.copy_(x)
        dist.all_reduce(z)
        e = float((z.float() - ref).abs().max().item()) / ref_max
        out["rccl"] = {"us": round(tr * 1e6, 1) if tr else None,
                       "busbw_GBps": round(busbw_gbps(n * 2, tr, world), 2) if tr else None,
                       "max_rel_err": round(max_vec([e])[0], 6)}
        del z
    del x, y, ref
    return out


CALIB_NOTE = "calibration mini-sweep of the tuner's candidates vs RCCL and the cost-model fit"


def calibrate_model(comm, timings, nbytes, esize, world, x, y, op, dist, max_over_ranks, rank, shared, verify,
                    with_rccl):
    """Mini-sweep of every correct tuner candidate at CALIB_SIZES (each result checked against the RCCL
    reference, which is elementwise, so a prefix of it is the reference of the prefix), next to RCCL's own
    allreduce of the same bytes: a flexar-vs-RCCL table across sizes from the driver's run (BASELINE #4).
    Then fit the cost model (utils/costfit.py) to the executor schedules' timings (these sizes plus the
    tuner's at the headline size) and report the fitted constants, the fit error and the schedule the
    FITTED model would pick at the headline size next to the tuner's winner ("cost-model-selected" priced
    with measured constants). Not installed: the timed region runs the tuner's pick. Times are max over
    ranks, so every rank fits the same rows. Every failure is agreed on before anything else collective."""
    import torch

    from allreduce_over_mpi_amd import _native as nv
    from allreduce_over_mpi_amd.utils.costfit import fit_model
    from allreduce_over_mpi_amd.utils.perf import busbw_gbps

    links = int(comm.topology().get("links", 0)) if not shared else 0
    # the model prices executor schedules over IPC only (not the copy engines or the message transport)
    model_specs = [s for s in timings if "+rccl" not in s and "+msg" not in s
                   and nv.model_features(s, world, float(nbytes), links, esize) is not None]
    rows = [{"spec": s, "bytes": nbytes, "us": timings[s] * 1e6, "esize": esize} for s in model_specs]
    table, wrong = [], []

    def t_of(fn, iters):
        failed = 0.0
        try:
            fn()
            torch.cuda.synchronize()
        except nv.FlexarError:
            failed = 1.0
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        try:
            if not failed:
                for _ in range(iters):
                    fn()
                torch.cuda.synchronize()
        except nv.FlexarError:
            failed = 1.0
        dt = max_over_ranks(time.perf_counter() - t0 + (1e9 if failed else 0.0))
        return None if dt >= 1e9 else dt / iters

    broken = None
    for b in CALIB_SIZES:
        n = b // esize
        if n >= x.numel():
            continue
        xv, yv = x[:n], y[:n]
        iters = max(5, min(50, int(2e8 // b)))
        # the latency protocols join at the sizes they are built for
        extra = [s for s in (["ll", "oneshot"] if b <= (1 << 20) else ["oneshot"] if b <= (8 << 20) else [])
                 if s not in timings]
        best, best_t = None, float("inf")
        for s in list(timings) + extra:
            # local first call + check (a failure on any rank is agreed on before anything collective)
            failed, err = 0.0, 0.0
            try:
                comm.all_reduce(xv, out=yv, op=op, algo=s)
                torch.cuda.synchronize()
                comm.check()
                ok, err = verify(yv, n)
                failed = 0.0 if ok else 0.5
            except Exception as e:  # noqa: BLE001 - reported in the JSON line
                log(rank, f"calibration: {s} at {b} B failed on this rank: {e}")
                failed = 1.0
            failed = max_over_ranks(failed)
            if failed:
                wrong.append(f"{s}@{b}" + (" (error)" if failed >= 1.0 else f" (rel err {err:.3g})"))
                if failed >= 1.0:  # the communicator may be inconsistent now: stop the sweep here
                    broken = f"{s} at {b} B"
                    break
                continue
            t = t_of(lambda: comm.all_reduce(xv, out=yv, op=op, algo=s), iters)
            if t is None:
                wrong.append(f"{s}@{b} (timed call failed)")
                broken = f"{s} at {b} B"
                break
            if "+rccl" not in s and nv.model_features(s, world, float(b), links, esize) is not None:
                rows.append({"spec": s, "bytes": b, "us": t * 1e6, "esize": esize})
            if t < best_t:
                best, best_t = s, t
        if broken:
            break
        row = {"bytes": b, "flexar_best": best, "flexar_us": round(best_t * 1e6, 1) if best else None,
               "flexar_busbw": round(busbw_gbps(b, best_t, world), 2) if best else None}
        if with_rccl:
            z = xv.clone()
            tr = t_of(lambda: dist.all_reduce(z), iters)
            row.update(rccl_us=round(tr * 1e6, 1) if tr else None,
                       rccl_busbw=round(busbw_gbps(b, tr, world), 2) if tr else None)
        table.append(row)
        log(rank, "calibration sweep", json.dumps(row))
    out = {"sweep_vs_rccl": table, "wrong": wrong or None, "broken": broken}
    try:
        fit = fit_model(rows, world, links)
    except ValueError as e:
        out["error"] = str(e)
        return out
    feats = {s: nv.model_features(s, world, float(nbytes), links, esize) for s in model_specs}
    theta = (fit["alpha_launch_us"], fit["alpha_sync_us"], 1.0 / fit["link_gbps"], 1.0 / fit["hbm_gbps"])
    pick = min(model_specs, key=lambda s: sum(f * t for f, t in zip(feats[s], theta)))
    best = min(timings, key=timings.get)
    out.update({"FLEXAR_MODEL": fit["FLEXAR_MODEL"], "rows": fit["rows"],
                "median_rel_err": round(fit["median_rel_err"], 3), "max_rel_err": round(fit["max_rel_err"], 3),
                "winner_agreement": round(fit["winner_agreement"], 2), "max_regret": round(fit["max_regret"], 3),
                "fitted_choice": pick, "fitted_choice_us": round(timings[pick] * 1e6, 1),
                "tuner_best": best, "tuner_best_us": round(timings[best] * 1e6, 1), "sizes": fit["sizes"]})
    log(rank, f"calibration: FLEXAR_MODEL={fit['FLEXAR_MODEL']} median rel err {out['median_rel_err']}, "
              f"fitted choice {pick} ({out['fitted_choice_us']} us) vs tuner best {best} ({out['tuner_best_us']} us)")
    return out


def parse_bytes(v: str) -> int:
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    v = v.strip().upper().rstrip("B")
    return int(float(v[:-1]) * mult[v[-1]]) if v and v[-1] in mult else int(float(v))


def run_sweep(comm, world, rank, dev, dtype, op, dist, max_over_ranks, lo, hi, with_rccl, timed_fn, sweep_out=""):
    """busbw vs bytes, flexar (the selector's 'auto' choice) vs RCCL - BASELINE config #4. Every size is also
    a correctness check: rank r's input is (i mod 251) + r, whose sum N (i mod 251) + N (N - 1) / 2 is exact in
    every dtype used here and computed locally (no reference collective on multi-GiB buffers)."""
    import torch

    from allreduce_over_mpi_amd.utils.perf import busbw_gbps

    es = torch.tensor([], dtype=dtype).element_size()
    rows = []
    for b in _x4(lo, hi):
        n = max(1, b // es)
        pat = torch.remainder(torch.arange(n, device=dev, dtype=torch.int32), 251)
        x = (pat + rank).to(dtype)
        want = (pat * world + world * (world - 1) // 2).to(torch.float32)
        del pat
        y = torch.empty_like(x)
        iters = max(3, min(50, int(2e8 // max(b, 1))))
        tf = timed_fn(lambda: comm.all_reduce(x, out=y, op=op), iters, 2)
        if tf is None:  # failed on some rank (agreed inside timed_fn): the next size starts clean
            _recover(comm)
        # integers up to 2^24 (fp32) / 2048 (fp16) / 256 (bf16) are exact, and so is every partial sum below them
        limit = {torch.float32: 1 << 24, torch.float16: 2048, torch.bfloat16: 256}.get(dtype, 0)
        exact = op == "sum" and 250 * world + world * (world - 1) // 2 <= limit
        ok = None
        if exact:  # every rank's result, agreed on by every rank
            ok = max_over_ranks(0.0 if tf is not None and torch.equal(y.float(), want) else 1.0) == 0.0
        row = {"bytes": n * es, "algo": comm.describe(n, dtype).split(" ")[0],
               "flexar_us": round(tf * 1e6, 2) if tf else None,
               "flexar_busbw": round(busbw_gbps(n * es, tf, world), 2) if tf else None, "correct": ok}
        del want
        if with_rccl and world > 1:
            tr = timed_fn(lambda: dist.all_reduce(x), iters, 2)
            row.update(rccl_us=round(tr * 1e6, 2) if tr else None,
                       rccl_busbw=round(busbw_gbps(n * es, tr, world), 2) if tr else None)
        rows.append(row)
        log(rank, "sweep", json.dumps(row))
        if rank == 0 and sweep_out:
            with open(sweep_out, "a") as f:
                f.write(json.dumps(dict(row, n_gpus=world, dtype=str(dtype).replace("torch.", ""))) + "\n")
        del x, y
    return {"rows": rows} if rows else {"rows": []}


if __name__ == "__main__":
    main()
