"""Device communicators over the native flexar runtime.

* :class:`Communicator` — one rank per process / per GPU (the production path).
  Bootstrap: every rank exports its workspace IPC handles, the bytes are
  all-gathered through ``torch.distributed`` (any backend: gloo or RCCL), then
  each rank maps its peers' workspaces. After that an allreduce is a single
  stream-ordered kernel launch with no host involvement — the reference's
  ``MPI_Allreduce_FT`` (allreduce_over_mpi/mpi_mod.hpp:1167-1221) on
  GPU-resident tensors.
* :class:`LocalGroup` — ``n`` ranks inside ONE process on ONE GPU, all ranks in
  one launch. Runs the complete multi-rank device protocol without IPC; used by
  the GPU test-suite and for calibration.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

from .. import _native as nv


def _raw_stream_fn():
    import torch

    f = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    return f if f is not None else (lambda dev: torch.cuda.current_stream(dev).cuda_stream)


_RAW_STREAM = None


def _stream_handle(stream=None, device: Optional[int] = None) -> int:
    """hipStream_t of ``stream``, else of the current stream of ``device`` (default: current device)."""
    global _RAW_STREAM
    if stream is not None:
        return int(stream.cuda_stream)
    if _RAW_STREAM is None:
        _RAW_STREAM = _raw_stream_fn()
    if device is None:
        import torch

        device = torch.cuda.current_device()
    return int(_RAW_STREAM(device))


# per-call enum lookups, memoised by the (hashable) dtype / op objects the callers pass
_DT_CODES: dict = {}
_OP_CODES: dict = {}


def _dt(dtype) -> int:
    c = _DT_CODES.get(dtype)  # torch dtypes are singletons: the memo holds at most one entry per dtype
    if c is None:
        c = _DT_CODES[dtype] = nv.dtype_code(dtype)
    return c


def _op(op) -> int:
    if type(op) is not str:  # ints pass through; other op objects are not memoised (unbounded identities)
        return nv.op_code(op)
    c = _OP_CODES.get(op)
    if c is None:
        c = _OP_CODES[op] = nv.op_code(op)
    return c


_ALGO_BYTES: dict = {None: None}


def _algo(algo: Optional[str]):
    b = _ALGO_BYTES.get(algo)
    if b is None and algo:
        b = algo.encode()
        if len(_ALGO_BYTES) < 256:  # specs are a small fixed vocabulary; never grow without bound
            _ALGO_BYTES[algo] = b
    return b


def _require_cuda(t, what="tensor"):
    if not t.is_cuda:
        raise nv.FlexarError(1, f"{what} must be a ROCm device tensor")
    if not t.is_contiguous():
        raise nv.FlexarError(1, f"{what} must be contiguous")


class Communicator:
    """flexar communicator for the calling rank of a ``torch.distributed`` group."""

    def __init__(self, group=None, device: Optional[int] = None, workspace_bytes: int = 0,
                 algo: Optional[str] = None, rank: Optional[int] = None, world_size: Optional[int] = None,
                 exchange=None, transport: Optional[str] = None):
        """``exchange(bytes) -> list[bytes]`` all-gathers the handle bytes (default: torch.distributed
        all_gather_object on ``group``; :func:`store_exchange` bootstraps from a c10d Store).

        ``transport`` (default FLEXAR_TRANSPORT or "auto"): "ipc" = peer workspaces mapped over HIP IPC,
        fail if that is impossible; "auto" = IPC, and if any rank cannot map its peers, every call runs
        over the message transport (RCCL send/recv + local executor segments, csrc/include/flexar/
        msg_plan.hpp) with the same FlexTree / ring / RHD schedules; "rccl" = IPC plus the message
        transport (algorithm suffix "+rccl")."""
        import torch
        import torch.distributed as dist

        self._lib = nv.lib()
        if rank is None or world_size is None:
            if dist.is_available() and dist.is_initialized():
                rank = dist.get_rank(group)
                world_size = dist.get_world_size(group)
            else:
                rank, world_size = 0, 1
        self.rank, self.world_size = int(rank), int(world_size)
        self.device = torch.cuda.current_device() if device is None else int(device)
        self.group = group
        self._h = ctypes.c_void_p()
        self._hi = 0
        self.retried = None  # why the first attempt of an auto-transport connect failed (it was retried)
        transport = transport or os.environ.get("FLEXAR_TRANSPORT", "auto")
        if transport not in ("auto", "ipc", "rccl"):
            raise nv.FlexarError(1, f"unknown transport {transport!r} (auto | ipc | rccl)")
        if self.world_size > 1 and exchange is None:
            def exchange(data: bytes):
                gathered = [None] * self.world_size
                dist.all_gather_object(gathered, data, group=group)
                return gathered
        # transport "auto": a failure every rank agreed on at connect or in the readiness gate (a HIP error
        # in the self-test, no verified protocol) closes the communicator collectively and builds it once
        # more in this process; the second failure is final
        attempts = 2 if transport == "auto" and self.world_size > 1 else 1
        for attempt in range(attempts):
            try:
                self._open(workspace_bytes, exchange, transport)
                break
            except nv.FlexarError as e:
                self.close()
                if attempt + 1 == attempts or not getattr(e, "agreed", False):
                    raise
                self.retried = str(e)
                nv.log_warn(f"rank {self.rank}: communicator creation failed on every rank ({e}); "
                            "closed collectively, building it once more")
        self._rccl_default = False
        self._rccl_group = None
        env_algo = os.environ.get("FLEXAR_ALGO", "")
        if algo or env_algo == "rccl":
            self.set_algo(algo or env_algo)

    @staticmethod
    def _agreed(err: "nv.FlexarError") -> "nv.FlexarError":
        """Mark an error every rank raises identically (after an exchange): the collective retry may run."""
        err.agreed = True
        return err

    def _phase(self, what: str):
        """Breadcrumb (+ stderr line under FLEXAR_PHASE_LOG=1) of a creation phase on this rank."""
        nv.phase("comm: " + what, self.rank, self.world_size)

    def _open(self, workspace_bytes, exchange, transport):
        """Create, export, connect and verify the native communicator (collective)."""
        import torch

        self._phase(f"create (workspace {int(workspace_bytes)} B, transport {transport})")
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            nv.check(self._lib.flexar_comm_create(self.rank, self.world_size, self.device, int(workspace_bytes),
                                                  ctypes.byref(h)), "comm_create")
        self._h = h
        self._hi = int(h.value or 0)  # the handle as an int, for the fast-call path
        self.selftest_failed = []
        self.selftest_notes = {}
        self.selftest_recovered = []
        self.selftest_flaky = []
        self.calibration = None
        self.transport_note = None
        self.host_page_note = None
        self._exchange = None
        self._regs = {}
        self._zc_ok = None  # zero-copy readiness: None = not checked yet (first register())
        self._zc_testing = False
        if self.world_size == 1:
            return
        hs = int(self._lib.flexar_handle_size())
        buf = ctypes.create_string_buffer(hs)
        nv.check(self._lib.flexar_comm_export(self._h, buf), "comm_export")
        self._exchange = exchange
        self._phase("handle exchange")
        allb = b"".join(exchange(bytes(buf.raw)))
        self._phase("connect (map every peer)")
        rc = self._lib.flexar_comm_connect(self._h, allb)
        # agreement round (also the barrier: everyone has mapped everyone before the first collective);
        # a rank that failed to map a peer must not leave the others waiting in a later collective
        msg = b"" if rc == 0 else f"{rc}:rank {self.rank}: {nv.last_error()}".encode()
        bad = [m.decode(errors="replace") for m in exchange(msg) if m]
        # no peer memory (a failed peer mapping = HIP error 3; no P2P path between the GPUs or ranks on
        # different hosts = unsupported 2) falls back to the message transport; settings mismatches
        # (invalid 1) stay errors
        mapping_only = bool(bad) and all(b.split(":", 1)[0] in ("2", "3") for b in bad)
        fallback = bool(bad) and transport == "auto" and mapping_only and self._lib.flexar_rccl_available()
        if bad and not fallback:
            err = nv.FlexarError(rc or 5, "comm_connect: " + "; ".join(b.split(":", 1)[1] for b in bad))
            raise self._agreed(err) if mapping_only else err  # settings mismatches would only fail again
        self._verify_host_page(exchange)
        if transport == "rccl" or fallback:
            self._phase("message transport (ncclCommInitRank)")
            self._init_msg(exchange)
            if fallback:
                nv.check(self._lib.flexar_comm_connect_msg_only(self._h), "connect_msg_only")
                self.transport_note = "IPC unavailable (" + "; ".join(b.split(":", 1)[1] for b in bad) + \
                                      "): every call runs over the RCCL message transport"
        self._phase("probe agreement")
        self._agree_probe(exchange)
        self._readiness(exchange)
        self._phase("calibration")
        self._calibrate(exchange)
        self._phase("ready")

    def _verify_host_page(self, exchange):
        """Is the teardown / agreement page (csrc/src/host_barrier.hpp) shared by every rank? Every rank wrote
        its mark into the page at connect; the exchange right after connect was the barrier, so the check is
        immediate: a rank whose page lacks a peer's mark (one container per rank, a private /dev/shm) says so,
        and then every rank drops the page - teardown parks exported buffers instead of waiting out the
        timeout, host agreements go to the bootstrap."""
        ok = ctypes.c_int(0)
        if self.topology().get("host_page"):
            nv.check(self._lib.flexar_comm_host_page_check(self._h, ctypes.byref(ok)), "host_page_check")
        rows = exchange(b"1" if ok.value else b"0")
        if all(r == b"1" for r in rows):
            self.host_page_note = None
            return
        nv.check(self._lib.flexar_comm_host_page_drop(self._h), "host_page_drop")
        self.host_page_note = ("host page not shared (no mark from rank(s) "
                               f"{[i for i, r in enumerate(rows) if r != b'1']}): close() agrees over the bootstrap "
                               "exchange instead (a close without it keeps this rank's workspace allocated)")
        if self.rank == 0:
            nv.log_warn(self.host_page_note)

    def _init_msg(self, exchange):
        """Create the RCCL communicator of the message transport (collective): rank 0's unique id is
        all-gathered through ``exchange``."""
        uid = ctypes.create_string_buffer(128)
        if self.rank == 0:
            nv.check(self._lib.flexar_rccl_unique_id(uid, 128), "rccl_unique_id")
        ids = exchange(bytes(uid.raw) if self.rank == 0 else b"")
        rc = self._lib.flexar_comm_init_msg(self._h, ids[0])
        bad = [m.decode(errors="replace") for m in exchange(b"" if rc == 0 else
                                                            f"rank {self.rank}: {nv.last_error()}".encode()) if m]
        if bad:
            raise nv.FlexarError(7, "message transport: " + "; ".join(bad))

    def _agree_probe(self, exchange):
        """Probe agreement (flexar_comm_probe_agree): every rank's link classes / link count / settings
        fingerprint are exchanged; the minimum link count is installed everywhere and a real disagreement
        (asymmetric link classes, different settings) fails on every rank with a message naming the ranks,
        instead of as a device watchdog timeout in the first collective."""
        blob = ctypes.create_string_buffer(int(self._lib.flexar_probe_blob_size()))
        nv.check(self._lib.flexar_comm_probe_export(self._h, blob), "probe_export")
        rc = self._lib.flexar_comm_probe_agree(self._h, b"".join(exchange(bytes(blob.raw))))
        if rc:  # deterministic on identical inputs: every rank fails the same way
            raise nv.FlexarError(rc, "comm_connect: " + nv.last_error())

    def _calibrate(self, exchange):
        """Connect-time calibration of the cost model (flexar_comm_calibrate; FLEXAR_CALIB = 0 | 1 (default:
        the cached constants of this node shape, else measure) | force): a few executor schedules timed on
        the real links, max over ranks, fitted and installed identically on every rank. If the ranks end up
        with different models (a rank failed mid-way), every rank falls back to the default model."""
        import json

        self.calibration = None
        mode = {"0": 0, "off": 0, "1": 1, "force": 2, "2": 2}.get(os.environ.get("FLEXAR_CALIB", "1"), 1)
        exchange(b"")  # start together: a rank still finishing the self-test must not trip the short watchdog
        buf = ctypes.create_string_buffer(1 << 14)
        rc = self._lib.flexar_comm_calibrate(self._h, mode, buf, 1 << 14)
        err = nv.last_error() if rc else ""
        h = int(self._lib.flexar_comm_model_hash(self._h)) if rc == 0 else 0
        rows = exchange(f"{rc}:{h}".encode())
        if len(set(rows)) != 1 or rc:
            nv.check(self._lib.flexar_comm_clear_error(self._h), "clear_error")
            nv.check(self._lib.flexar_comm_reset_model(self._h), "reset_model")
            self.calibration = {"source": "disagreed", "error": err or None,
                                "ranks": [r.decode(errors="replace") for r in rows]}
            exchange(b"")
            return
        try:
            self.calibration = json.loads(buf.value.decode() or "{}")
        except ValueError:
            self.calibration = {"source": "unparsed", "raw": buf.value.decode(errors="replace")}

    def _readiness(self, exchange):
        """Connect-time self-test (flexar_comm_selftest): every protocol family runs exact integer
        allreduces on the real links; a family that failed on ANY rank is disabled on every rank, and
        calls move to a verified one (ll -> oneshot, fence -> +wt -> dma). FLEXAR_SELFTEST=0 skips it."""
        self.selftest_failed: list[str] = []
        if os.environ.get("FLEXAR_SELFTEST", "1") == "0":
            return
        # FLEXAR_SELFTEST_SKEW="RANK:MS" (tests): that rank starts the first family MS late, past its peers'
        # watchdog - the transient failure the retry below must absorb
        skew = os.environ.get("FLEXAR_SELFTEST_SKEW", "")
        late_ms = float(skew.split(":")[1]) if skew.count(":") == 1 and int(skew.split(":")[0]) == self.rank else 0.0

        def run(fam):
            """One family's exact allreduces, started together (a barrier first: a rank that arrives seconds
            late - e.g. still finishing RCCL set-up - would otherwise trip its peers' short watchdog and shift
            every later family out of step); returns the families that failed on ANY rank.

            A HIP error on a rank fails the family there, with the error named (flexar_comm_selftest_note), and
            the downgrade chain goes on; only an error that left the device unusable (rc != 0) ends creation,
            with every rank's message, on every rank."""
            nonlocal late_ms
            self._phase(f"self-test {','.join(nv.family_names(fam))}")
            exchange(b"")
            if late_ms:
                import time

                time.sleep(late_ms / 1000.0)
                late_ms = 0.0
            failed = ctypes.c_uint32(0)
            rc = self._lib.flexar_comm_selftest(self._h, fam, ctypes.byref(failed))
            note = nv.last_error() if rc else self._selftest_note()
            msg = f"{rc}:{failed.value}:{note}".encode()
            rows = [m.decode(errors="replace").split(":", 2) for m in exchange(msg)]  # also the barrier
            errs = [f"rank {r}: {e}" for r, (c, _, e) in enumerate(rows) if c != "0"]
            if errs:
                # the device is unusable on those ranks (a sticky HIP error): a retry could not run either
                raise nv.FlexarError(3, "self-test: " + "; ".join(errs))
            m = 0
            for r, (_, f, e) in enumerate(rows):
                m |= int(f)
                if e:
                    self.selftest_notes.setdefault(r, []).append(e)
            if m:
                if self.rank == 0:
                    nv.log_warn("self-test: family " + ",".join(nv.family_names(m)) + " failed: " +
                                "; ".join(f"rank {r}: {e}" for r, (_, f, e) in enumerate(rows) if e))
                # every rank has finished every call of this family (the exchange above): a launch that never
                # ran left its rank's epochs behind, so the protocol state is reset on every rank, and nobody
                # starts the next family before every rank has reset
                nv.check(self._lib.flexar_comm_resync(self._h), "resync")
                exchange(b"")
            return m

        mask = 0
        for fam in nv.FAMILIES.values():
            mask |= run(fam)
        # Every failed family runs a second time. A broken protocol fails again (families a communicator
        # cannot run at all, e.g. peer-memory ones without IPC mappings, fail at once without launching
        # anything). One that passes the second time is kept only when ranks share a GPU, where a rank
        # descheduled past its peers' watchdog is expected; with one GPU per rank a family that failed once
        # is a bug signal and stays disabled (selftest_policy).
        self.selftest_recovered = []
        self.selftest_flaky = []
        if mask:
            again = 0
            for fam in nv.FAMILIES.values():
                if mask & fam:
                    again |= run(fam)
            local_shared = shares_gpu(self.topology(), self.rank)
            shared_any = any(r == b"1" for r in exchange(b"1" if local_shared else b"0"))
            mask, recovered, flaky = selftest_policy(mask, again, shared_any)
            self.selftest_recovered = nv.family_names(recovered)
            self.selftest_flaky = nv.family_names(flaky)
        if mask:
            nv.check(self._lib.flexar_comm_set_disabled(self._h, mask), "set_disabled")
            self.selftest_failed = nv.family_names(mask)
            exchange(b"")  # nobody issues a production call before every rank installed the mask
            tested = sum(nv.FAMILIES[n] for n in self.topology()["selftested"].split(",") if n in nv.FAMILIES)
            if tested & ~mask == 0:
                raise self._agreed(nv.FlexarError(2, "no device protocol passed the connect-time self-test on this "
                                                     "node: " + "; ".join(f"rank {r}: {' / '.join(v)}"
                                                                          for r, v in self.selftest_notes.items())))

    def _selftest_note(self) -> str:
        b = ctypes.create_string_buffer(1024)
        self._lib.flexar_comm_selftest_note(self._h, b, 1024)
        return b.value.decode(errors="replace")

    def host_agree_max(self, value: int) -> int:
        """Collective: the maximum of ``value`` (0 .. 2**64 - 1) over the ranks, through the communicator's
        host shared-memory page - no device call, no bootstrap round trip. Raises
        FlexarError when the communicator has no page (single rank, in-process group)."""
        return self._host_agree(value, 0)

    def host_agree_or(self, value: int) -> int:
        """Collective: the bitwise OR of ``value`` over the ranks (see :meth:`host_agree_max`)."""
        return self._host_agree(value, 1)

    def _host_agree(self, value: int, op: int) -> int:
        out = ctypes.c_uint64(0)
        nv.check(self._lib.flexar_comm_host_agree(self._h, int(value), op, ctypes.byref(out)), "host_agree")
        return int(out.value)

    def topology(self) -> dict:
        """Connect-time probe: per-peer PCI bus id, device, link class and hop count; self-test state."""
        import json

        b = ctypes.create_string_buffer(1 << 14)
        nv.check(self._lib.flexar_comm_topology(self._h, b, 1 << 14), "comm_topology")
        return json.loads(b.value.decode())

    def predict_us(self, spec: str, nbytes: float) -> float:
        """Cost-model time of ``spec`` ("auto" = the model's choice) for ``nbytes`` on this node's probed links."""
        v = self._lib.flexar_comm_predict_us(self._h, spec.encode(), float(nbytes))
        if v < 0:
            raise nv.FlexarError(1, nv.last_error())
        return float(v)

    def recommended_bucket_bytes(self, efficiency: float = 0.9, zero_copy: bool = False) -> int:
        """Gradient-bucket size for DDP / FSDP on this node (``DDP(bucket_cap_mb=b / 2**20)``): the smallest
        size whose allreduce the calibrated selector prices at ``efficiency`` of its 1 GiB bandwidth
        (utils/perf.py recommend_bucket_bytes). ``zero_copy``: price the registered-buffer form the backend
        and the DDP hook run on persistent buckets. Identical on every rank (the model is agreed on)."""
        from ..utils.perf import recommend_bucket_bytes

        if self.world_size < 2:
            return 1 << 20
        spec = "flat+zc+push" if zero_copy else "auto"
        return recommend_bucket_bytes(lambda b: self.predict_us(spec, b), efficiency)

    def calibrate(self, rows, install: bool = True) -> dict:
        """Fit the cost model to measured rows ({"spec", "bytes", "us"}: ``autotune``'s or
        tools/flexar_tune.py's) on this node's probed link count, and install it (every rank must pass the
        same rows, e.g. max-over-ranks timings). Returns the fit (utils/costfit.py)."""
        from ..utils.costfit import fit_model

        links = int(self.topology().get("links", 0)) if self.world_size > 1 else 0
        fit = fit_model(rows, self.world_size, links)
        if install:
            nv.check(self._lib.flexar_comm_set_model(self._h, fit["alpha_launch_us"], fit["alpha_sync_us"],
                                                     fit["link_gbps"], fit["hbm_gbps"], links), "set_model")
        return fit

    # ------------------------------------------------------------------ config
    def set_algo(self, spec: str):
        """Default algorithm spec (see README); ``"rccl"`` routes allreduces to RCCL (comparator / fallback)."""
        self._rccl_default = spec == "rccl"
        if not self._rccl_default:
            nv.check(self._lib.flexar_comm_set_algo(self._h, spec.encode()), "set_algo")

    def _rccl_all_reduce(self, tensor, op, out, scale):
        """FLEXAR_ALGO=rccl: the vendor collective on an RCCL group of the same ranks."""
        import torch.distributed as dist

        if self._rccl_group is None:
            if self.group is None and dist.get_backend() == "nccl":
                self._rccl_group = dist.group.WORLD
            elif self.group is not None and dist.get_backend(self.group) == "nccl":
                self._rccl_group = self.group
            else:
                self._rccl_group = dist.new_group(ranks=dist.get_process_group_ranks(self.group or dist.group.WORLD),
                                                  backend="nccl")
        dst = tensor if out is None else out.copy_(tensor)
        ops = {"sum": dist.ReduceOp.SUM, "avg": dist.ReduceOp.AVG, "max": dist.ReduceOp.MAX,
               "min": dist.ReduceOp.MIN, "prod": dist.ReduceOp.PRODUCT, "band": dist.ReduceOp.BAND,
               "bor": dist.ReduceOp.BOR, "bxor": dist.ReduceOp.BXOR}
        dist.all_reduce(dst, op=ops[op], group=self._rccl_group)
        if scale != 1.0:
            dst.mul_(scale)
        return dst

    def set_grid(self, grid: int):
        nv.check(self._lib.flexar_comm_set_grid(self._h, int(grid), 0), "set_grid")

    def set_xfer_chunk(self, elems: int):
        """Executor work split of large spans: see LocalGroup.set_xfer_chunk. Collective: producer and consumer
        workgroups must split a span the same way on every rank, so the ranks exchange the value first and
        a mismatch raises on every rank, leaving the setting unchanged (a silent mismatch would
        misassign elements or hang)."""
        elems = int(elems)
        if self.world_size > 1 and self._exchange is not None:
            rows = [r.decode() for r in self._exchange(str(elems).encode())]
            if len(set(rows)) != 1:
                raise self._agreed(nv.FlexarError(1, f"set_xfer_chunk: ranks disagree ({rows})"))
        nv.check(self._lib.flexar_comm_set_xfer_chunk(self._h, elems), "set_xfer_chunk")

    def set_tune_table(self, text: str):
        """Install a measured "nranks bytes spec" table (FLEXAR_TUNE_FILE format); "" = cost model."""
        nv.check(self._lib.flexar_comm_set_tune_table(self._h, text.encode()), "set_tune_table")

    def autotune(self, **kw):
        """Measure the candidate schedules on this node and install the winners (collective);
        see :func:`allreduce_over_mpi_amd.parallel.autotune.autotune`."""
        from .autotune import autotune

        return autotune(self, **kw)

    def describe(self, count: int, dtype) -> str:
        b = ctypes.create_string_buffer(512)
        nv.check(self._lib.flexar_comm_describe(self._h, int(count), nv.dtype_code(dtype), b, 512), "describe")
        return b.value.decode()

    def last_spec(self) -> str:
        """The schedule the last allreduce on this communicator ran, after the zero-copy decision (``describe``
        gives the plan before it: registered buffers may turn the flat choice into ``+zc+push``); "" before any."""
        b = ctypes.create_string_buffer(256)
        nv.check(self._lib.flexar_comm_last_spec(self._h, b, 256), "last_spec")
        return b.value.decode()

    def check(self):
        nv.check(self._lib.flexar_comm_check(self._h), "comm_check")

    def clear_error(self):
        """Forget a recorded watchdog timeout (call on every rank after all of them synchronised)."""
        nv.check(self._lib.flexar_comm_clear_error(self._h), "comm_clear_error")

    def stats(self) -> dict:
        """Call/byte counters; per-algorithm device time when FLEXAR_PROFILE=1 (synchronises those events)."""
        import json

        b = ctypes.create_string_buffer(1 << 16)
        nv.check(self._lib.flexar_comm_stats(self._h, b, 1 << 16), "comm_stats")
        return json.loads(b.value.decode())

    # ------------------------------------------------------------------ registered buffers
    def register(self, tensor) -> int:
        """Register a device buffer for zero-copy allreduce (algorithm suffix "+zc", e.g. "flat+zc"): the
        flat schedule then reads every peer's input and output straight over IPC, with no staging copies.
        Collective: every rank registers its corresponding tensor (same byte size), in the same order.
        The communicator holds a reference until :meth:`deregister`. A "+zc" call takes tensors that lie
        inside registrations, at the same offset on every rank (DDP buckets, FSDP flat parameters).

        The first registration runs the zero-copy readiness check (:meth:`_zc_selftest`, like the
        connect-time self-test of the staging protocols): if the peers' buffers do not read back exactly
        on this node, every rank raises here and callers keep the staging schedules. The peers map the
        whole allocation holding the tensor; allocations above 1 GiB are refused (FLEXAR_REG_MAX_ALLOC;
        docs/DESIGN.md §17), so allocate large registered buffers on their own.

        Once registered, calls with no named spec switch to zero copy by themselves (FLEXAR_ZC_AUTO):
        allreduce when the cost model prefers it, reduce-scatter / all-gather / all-to-all always."""
        _require_cuda(tensor)
        if self.world_size > 1 and self._zc_ok is None:
            self._zc_ok = False  # (re-entry from the self-test's own registration)
            self._zc_ok = self._zc_selftest()
        if self.world_size > 1 and self._zc_ok is False and not self._zc_testing:
            raise nv.FlexarError(2, "register: zero copy failed its readiness check on this node "
                                    "(peer buffers did not read back exactly); use the staging schedules")
        return self._register(tensor)

    def _zc_selftest(self) -> bool:
        """Exact integer allreduces over a registered scratch buffer with both zero-copy forms, three
        consecutive calls each (the calls' hand-offs and the peers' reads of freshly written buffers are
        what could fail across devices). Collective; True when every rank got exact sums."""
        import torch

        if os.environ.get("FLEXAR_SELFTEST", "1") == "0":
            return True
        n = 65536 + 77
        # the scratch allocation is agreed on before anything collective: a rank that cannot allocate must
        # not leave its peers inside the registration's exchanges while it waits in the final agreement
        try:
            buf = torch.empty(2 * n + 64, dtype=torch.int32, device=f"cuda:{self.device}")
            x, y = buf[:n], buf[n + 64:]
            idx = torch.arange(n, dtype=torch.int32, device=buf.device) % 1009
            have = b"1"
        except Exception:  # noqa: BLE001 - out of memory or a device error on this rank
            have = b"0"
        if any(r != b"1" for r in self._exchange(have)):
            return False
        ok = True
        self._zc_testing = True
        rid = None
        # every later failure on this rank (registration, calls, checks) is a "no" in the agreement below,
        # which every rank reaches: the registration and the calls are collective with their own agreements
        try:
            rid = self._register(buf)
            w = self.world_size
            for spec in ("flat+zc+push", "flat+zc"):
                for call in range(3):
                    x.copy_(idx * (self.rank + 1) + call)
                    self.all_reduce(x, out=y, algo=spec)
                    want = idx * (w * (w + 1) // 2) + call * w
                    ok = ok and bool(torch.equal(y, want))
            self.check()
        except Exception:  # noqa: BLE001 - any failure on this rank is a "no" in the agreement
            ok = False
        finally:
            self._zc_testing = False
        rows = self._exchange(b"1" if ok else b"0")  # also the barrier: no rank is inside a test call
        passed = all(r == b"1" for r in rows)
        if not passed:
            self.clear_error()  # a timed-out test call must not fail the next production call
        if rid is not None:
            try:
                self.deregister(rid)
            except nv.FlexarError:
                pass
        return passed

    def _register(self, tensor) -> int:
        nbytes = tensor.numel() * tensor.element_size()
        blob = ctypes.create_string_buffer(int(self._lib.flexar_reg_handle_size()))
        rc = self._lib.flexar_reg_export(self._h, tensor.data_ptr(), nbytes, blob)
        err = nv.last_error() if rc else ""
        rows = [bytes(blob.raw) if rc == 0 else b""]
        if self.world_size > 1:
            rows = self._exchange(rows[0])
            if any(not r for r in rows):  # every rank agrees before anything is mapped
                raise nv.FlexarError(rc or 1, f"register: export failed on rank(s) "
                                              f"{[i for i, r in enumerate(rows) if not r]} {err}".rstrip())
        rid = ctypes.c_int(0)
        rc = self._lib.flexar_reg_open(self._h, tensor.data_ptr(), nbytes, b"".join(rows), ctypes.byref(rid))
        msg = b"" if rc == 0 else f"rank {self.rank}: {nv.last_error()}".encode()
        bad = [m.decode(errors="replace") for m in (self._exchange(msg) if self.world_size > 1 else [msg]) if m]
        if bad:
            if rc == 0:
                self._lib.flexar_reg_close(self._h, rid.value)
            raise nv.FlexarError(rc or 1, "register: " + "; ".join(bad))
        self._regs[rid.value] = tensor
        self._prune_regs()
        return rid.value

    def _prune_regs(self):
        """Drop the references of registrations the native side replaced (a newer registration contained
        them, or their allocation was freed and reused): they must not keep dead tensors alive."""
        ids = (ctypes.c_int * 4096)()
        k = self._lib.flexar_reg_ids(self._h, ids, 4096)
        live = set(ids[:min(k, 4096)])
        for old in [r for r in self._regs if r not in live]:
            del self._regs[old]

    def register_many(self, tensors) -> list:
        """:meth:`register` for several tensors with one handle exchange and one agreement round (every
        rank passes its corresponding tensors in the same order). Returns the registration ids."""
        tensors = list(tensors)
        if self.world_size == 1 or not tensors:
            return [self.register(t) for t in tensors]
        if self._zc_ok is None:
            self._zc_ok = False
            self._zc_ok = self._zc_selftest()
        if self._zc_ok is False:
            raise nv.FlexarError(2, "register: zero copy failed its readiness check on this node "
                                    "(peer buffers did not read back exactly); use the staging schedules")
        hs = int(self._lib.flexar_reg_handle_size())
        blobs, err = [], ""
        for t in tensors:
            _require_cuda(t)
            b = ctypes.create_string_buffer(hs)
            if self._lib.flexar_reg_export(self._h, t.data_ptr(), t.numel() * t.element_size(), b):
                err = nv.last_error()
                break
            blobs.append(bytes(b.raw))
        rows = self._exchange(b"".join(blobs) if not err else b"")
        if any(len(r) != hs * len(tensors) for r in rows):
            raise nv.FlexarError(1, f"register: export failed on rank(s) "
                                    f"{[i for i, r in enumerate(rows) if len(r) != hs * len(tensors)]} {err}".rstrip())
        ids, msg = [], b""
        for k, t in enumerate(tensors):
            all_k = b"".join(r[k * hs:(k + 1) * hs] for r in rows)
            rid = ctypes.c_int(0)
            if self._lib.flexar_reg_open(self._h, t.data_ptr(), t.numel() * t.element_size(), all_k, ctypes.byref(rid)):
                msg = f"rank {self.rank}: {nv.last_error()}".encode()
                break
            ids.append(rid.value)
        bad = [m.decode(errors="replace") for m in self._exchange(msg) if m]
        if bad:
            for rid in ids:
                self._lib.flexar_reg_close(self._h, rid)
            raise nv.FlexarError(1, "register: " + "; ".join(bad))
        for rid, t in zip(ids, tensors):
            self._regs[rid] = t
        self._prune_regs()
        return ids

    def deregister(self, rid: int):
        """Drop a registration (every rank, once the calls using it have completed)."""
        nv.check(self._lib.flexar_reg_close(self._h, int(rid)), "deregister")
        self._regs.pop(int(rid), None)

    # ------------------------------------------------------------------ collectives
    def all_reduce(self, tensor, op="sum", out=None, algo: Optional[str] = None, scale: float = 1.0, stream=None):
        """Allreduce ``tensor`` (in place unless ``out`` is given). Returns the result tensor."""
        _require_cuda(tensor)
        if algo == "rccl" or (algo is None and self._rccl_default):
            return self._rccl_all_reduce(tensor, op, out, scale)
        dst = tensor if out is None else out
        if out is not None:
            _require_cuda(out, "out")
            if out.numel() != tensor.numel() or out.dtype != tensor.dtype:
                raise nv.FlexarError(1, "out must match tensor in size and dtype")
        args = (tensor.data_ptr(), dst.data_ptr(), tensor.numel(), _dt(tensor.dtype), _op(op),
                _stream_handle(stream, self.device), _algo(algo))
        if nv.FAST is not None:
            rc = nv.FAST.ar(nv.AR, self._hi, *args, float(scale))
        else:
            rc = self._lib.flexar_allreduce_ex(self._h, *args, float(scale))
        if rc:
            nv.check(rc, "allreduce")
        return dst

    def all_reduce_fp8(self, tensor, op="avg", out=None, wire: str = "e4m3", algo: Optional[str] = None, stream=None,
                       amax_parts=None):
        """Compressed allreduce of an fp32 / bf16 / fp16 ``tensor`` with OCP fp8 on the links (BASELINE
        config #5): one amax pass (``fp8_amax``, 256 per-workgroup partials, device-resident), then ONE
        executor launch that derives the pre-scale s = fp8_max / (N * global amax) from every rank's amax,
        quantises each contribution with it inside the first transfer, sums in fp32 and writes the result
        / s in the tensor's dtype inside the last. All ranks get identical results. In place unless ``out``.
        ``wire="mx_e4m3"`` / ``"mx_e5m2"``: the OCP MX form - one e8m0 scale per 32-element block, computed in
        the same single launch, so no amax pass (docs/DESIGN.md §9.2)."""
        from ..ops.quant import fp8_amax

        if wire in ("mx_e4m3", "mx_e5m2"):  # OCP MX block scales: computed inside the executor, no amax pass
            return self.all_reduce(tensor, op, out=out, algo=(algo or "flat+pull") + "+mx" + wire[3:], stream=stream)
        _require_cuda(tensor)
        dst = tensor if out is None else out
        if out is not None:
            _require_cuda(out, "out")
            if out.numel() != tensor.numel() or out.dtype != tensor.dtype:
                raise nv.FlexarError(1, "out must match tensor in size and dtype")
        if amax_parts is None:
            amax_parts = fp8_amax(tensor, stream=stream)
        wd = {"e4m3": nv.DTYPES["fp8_e4m3"], "e5m2": nv.DTYPES["fp8_e5m2"]}[wire]
        rc = self._lib.flexar_allreduce_fp8(self._h, tensor.data_ptr(), dst.data_ptr(), tensor.numel(),
                                            _dt(tensor.dtype), _op(op), _stream_handle(stream, self.device), wd,
                                            amax_parts.data_ptr(), _algo(algo))
        if rc:
            nv.check(rc, "allreduce_fp8")
        return dst

    def reduce_scatter(self, input, output, op="sum", algo: Optional[str] = None, stream=None):
        """``output`` (m elements) = this rank's reduced block of ``input`` (world_size * m elements)."""
        _require_cuda(input)
        _require_cuda(output, "output")
        if input.numel() != output.numel() * self.world_size or input.dtype != output.dtype:
            raise nv.FlexarError(1, "input must hold world_size * output.numel() elements of output's dtype")
        args = (input.data_ptr(), output.data_ptr(), output.numel(), _dt(output.dtype), _op(op),
                _stream_handle(stream, self.device), _algo(algo))
        rc = nv.FAST.rs(nv.RS, self._hi, *args) if nv.FAST is not None else \
            self._lib.flexar_reduce_scatter(self._h, *args)
        if rc:
            nv.check(rc, "reduce_scatter")
        return output

    def all_gather(self, input, output, algo: Optional[str] = None, stream=None):
        """``output`` (world_size * m elements) = concatenation of every rank's ``input`` (m elements)."""
        _require_cuda(input)
        _require_cuda(output, "output")
        if output.numel() != input.numel() * self.world_size or input.dtype != output.dtype:
            raise nv.FlexarError(1, "output must hold world_size * input.numel() elements of input's dtype")
        args = (input.data_ptr(), output.data_ptr(), input.numel(), _dt(input.dtype),
                _stream_handle(stream, self.device), _algo(algo))
        rc = nv.FAST.ag(nv.AG, self._hi, *args) if nv.FAST is not None else \
            self._lib.flexar_all_gather(self._h, *args)
        if rc:
            nv.check(rc, "all_gather")
        return output

    def all_to_all(self, input, output, stream=None, algo: Optional[str] = None):
        """Equal-split all-to-all (expert parallelism): block p of ``input`` (world_size blocks) goes to
        rank p; block q of ``output`` comes from rank q. One direct exchange over all links; ``algo``
        "flat+zc" writes straight into the peers' registered ``output`` (no staging)."""
        _require_cuda(input)
        _require_cuda(output, "output")
        if input.numel() != output.numel() or input.dtype != output.dtype or input.numel() % self.world_size:
            raise nv.FlexarError(1, "input/output must have equal size (a multiple of world_size) and dtype")
        nv.check(self._lib.flexar_all_to_all_ex(self._h, input.data_ptr(), output.data_ptr(),
                                                input.numel() // self.world_size, nv.dtype_code(input.dtype),
                                                _stream_handle(stream), _algo(algo)), "all_to_all")
        return output

    def broadcast(self, tensor, root: int = 0, out=None, algo: Optional[str] = None, stream=None):
        """Broadcast ``tensor`` of rank ``root`` (in place unless ``out`` is given) to every rank."""
        _require_cuda(tensor)
        dst = tensor if out is None else out
        if out is not None:
            _require_cuda(out, "out")
            if out.numel() != tensor.numel() or out.dtype != tensor.dtype:
                raise nv.FlexarError(1, "out must match tensor in size and dtype")
        nv.check(self._lib.flexar_broadcast(self._h, tensor.data_ptr(), dst.data_ptr(), tensor.numel(),
                                            nv.dtype_code(tensor.dtype), int(root), _stream_handle(stream),
                                            algo.encode() if algo else None), "broadcast")
        return dst

    def close(self, collective: bool = True):
        """Tear the communicator down. Collective (every rank, in the same order, like creation): the
        library drains this rank's calls, agrees with every peer that all calls have finished, closes the
        peer mappings (workspaces and registrations), agrees that every rank has unmapped, and only then
        frees (flexar_comm_destroy). ``collective=False`` (garbage collection) skips the agreements and
        leaves this rank's exported buffers allocated until the process exits."""
        if getattr(self, "_h", None) is not None and self._h.value:
            agree_fn = self._teardown_agreement() if collective else None
            self._hi = 0
            h, self._h = self._h, ctypes.c_void_p()
            self._regs = {}
            if not collective:
                rc = self._lib.flexar_comm_destroy_local(h)
            elif agree_fn is not None:
                rc = self._lib.flexar_comm_destroy_agreed(h, agree_fn, None)
            else:
                rc = self._lib.flexar_comm_destroy(h)
            if rc and collective:
                nv.log_warn(f"rank {self.rank}: close: {nv.last_error()}")

    def _teardown_agreement(self):
        """The two teardown agreements over the bootstrap exchange, for a communicator whose ranks found at
        connect that they share no host page (one container per rank, a private /dev/shm: every rank dropped it
        together, _verify_host_page). The library calls the returned barrier where the page's agreements would
        be, so the workspace is freed rather than parked. None otherwise: with the page the library
        agrees by itself, and a page dropped later by one rank's timed-out agreement is not an agreed state (its
        peers would not join an exchange), so that close parks and says so."""
        if self.world_size == 1 or self._exchange is None or not self.host_page_note:
            return None
        exchange = self._exchange

        def barrier(_ctx):
            try:
                exchange(b"")
                return 1
            except Exception:  # noqa: BLE001 - a failed agreement parks the workspace (reported by the library)
                return 0

        self._agree_cb = nv.AGREE_FN(barrier)  # kept alive for the duration of the destroy call
        return self._agree_cb

    def __del__(self):
        try:
            self.close(collective=False)  # GC order differs per rank: never wait for peers here
        except Exception:
            pass


def shares_gpu(topology: dict, rank: int) -> bool:
    """True when some peer of ``rank`` runs on the same device (the probe's "same-device" link class)."""
    return any(p["link"] == "same-device" for p in topology["peers"] if p["rank"] != rank)


def selftest_policy(first: int, second: int, shared_gpu: bool, mode: Optional[str] = None):
    """Families disabled after the connect-time self-test: ``first`` failed the first pass on some rank,
    ``second`` (a subset of them) failed again. Returns (disabled, recovered, flaky):
    * ranks sharing a GPU (``shared_gpu``: any rank has a peer on its own device): a family that passed the
      second time is kept (``recovered``) - a rank descheduled past its peers' watchdog is expected there;
    * one GPU per rank: it is disabled anyway (``flaky``) - an intermittent failure of a protocol on
      dedicated GPUs is a bug signal (e.g. a cross-device visibility problem), never descheduling.
    FLEXAR_SELFTEST_RETRY=keep | disable overrides the choice (``mode``)."""
    mode = mode if mode is not None else os.environ.get("FLEXAR_SELFTEST_RETRY", "")
    passed_again = first & ~second
    keep = shared_gpu if mode not in ("keep", "disable") else mode == "keep"
    if keep:
        return second, passed_again, 0
    return first, 0, passed_again


def store_exchange(store, rank: int, world_size: int, prefix: str = "flexar"):
    """An ``exchange`` callable over a c10d Store: every call is one all-gather round."""
    state = {"round": 0}

    def ex(data: bytes):
        rnd = state["round"]
        state["round"] += 1
        store.set(f"{prefix}/{rnd}/{rank}", data)
        return [bytes(store.get(f"{prefix}/{rnd}/{r}")) for r in range(world_size)]

    return ex


def file_exchange(directory: str, rank: int, world_size: int, prefix: str = "flexar", timeout_s: float = 300.0):
    """An ``exchange`` callable over a shared directory (no torch.distributed, no MPI): rank r writes
    ``<prefix>.<round>.<r>`` atomically (write + rename) and polls for every other rank's file.
    SURVEY.md §7.2 bootstrap option "env + file rendezvous"; the directory must be fresh per job."""
    import time

    state = {"round": 0}
    os.makedirs(directory, exist_ok=True)

    def ex(data: bytes):
        rnd = state["round"]
        state["round"] += 1
        path = os.path.join(directory, f"{prefix}.{rnd}.{rank}")
        with open(path + ".tmp", "wb") as f:
            f.write(data)
        os.replace(path + ".tmp", path)
        out, t0 = [], time.monotonic()
        for r in range(world_size):
            p = os.path.join(directory, f"{prefix}.{rnd}.{r}")
            while not os.path.exists(p):
                if time.monotonic() - t0 > timeout_s:
                    raise TimeoutError(f"file rendezvous: rank {r} never wrote {p}")
                time.sleep(0.005)
            with open(p, "rb") as f:
                out.append(f.read())
        return out

    return ex


class LocalGroup:
    """``nranks`` flexar ranks on one GPU in one process (single-launch group execution)."""

    def __init__(self, nranks: int, device: Optional[int] = None, workspace_bytes: int = 64 << 20):
        import torch

        self._lib = nv.lib()
        self.nranks = int(nranks)
        self.device = torch.cuda.current_device() if device is None else int(device)
        arr = (ctypes.c_void_p * self.nranks)()
        with torch.cuda.device(self.device):
            nv.check(self._lib.flexar_group_create(self.nranks, self.device, int(workspace_bytes), arr), "group_create")
        self._comms = arr

    def set_grid(self, grid: int):
        for r in range(self.nranks):
            nv.check(self._lib.flexar_comm_set_grid(self._comms[r], int(grid), 0), "set_grid")

    def set_xfer_chunk(self, elems: int):
        """Executor work split of large spans: 0 = per-workgroup slices, else round-robin chunks of ``elems``
        elements (a multiple of 8192; device_exec.hpp DevCtx::ichunk)."""
        for r in range(self.nranks):
            nv.check(self._lib.flexar_comm_set_xfer_chunk(self._comms[r], int(elems)), "set_xfer_chunk")

    def describe(self, count: int, dtype, rank: int = 0) -> str:
        b = ctypes.create_string_buffer(512)
        nv.check(self._lib.flexar_comm_describe(self._comms[rank], int(count), nv.dtype_code(dtype), b, 512),
                 "describe")
        return b.value.decode()

    def all_reduce(self, tensors: Sequence, op="sum", outs: Optional[Sequence] = None, algo: Optional[str] = None,
                   scale: float = 1.0, stream=None):
        if len(tensors) != self.nranks:
            raise nv.FlexarError(1, "need one tensor per rank")
        for t in tensors:
            _require_cuda(t)
        outs = list(tensors) if outs is None else list(outs)
        ins = (ctypes.c_void_p * self.nranks)(*[t.data_ptr() for t in tensors])
        ous = (ctypes.c_void_p * self.nranks)(*[t.data_ptr() for t in outs])
        rc = self._lib.flexar_group_allreduce(self._comms, self.nranks, ins, ous, tensors[0].numel(),
                                              nv.dtype_code(tensors[0].dtype), nv.op_code(op), _stream_handle(stream),
                                              algo.encode() if algo else None, float(scale))
        nv.check(rc, "group_allreduce")
        return outs

    def all_reduce_fp8(self, tensors: Sequence, op="avg", outs: Optional[Sequence] = None, wire: str = "e4m3",
                       stream=None):
        """fp8-wire allreduce of every rank of the group in one launch (see Communicator.all_reduce_fp8)."""
        from ..ops.quant import fp8_amax

        if wire in ("mx_e4m3", "mx_e5m2"):
            return self.all_reduce(tensors, op, outs=outs, algo="flat+pull+mx" + wire[3:], stream=stream)
        outs = list(tensors) if outs is None else list(outs)
        parts = [fp8_amax(t, stream=stream) for t in tensors]
        ins = (ctypes.c_void_p * self.nranks)(*[t.data_ptr() for t in tensors])
        ous = (ctypes.c_void_p * self.nranks)(*[t.data_ptr() for t in outs])
        amx = (ctypes.c_void_p * self.nranks)(*[p.data_ptr() for p in parts])
        wd = {"e4m3": nv.DTYPES["fp8_e4m3"], "e5m2": nv.DTYPES["fp8_e5m2"]}[wire]
        nv.check(self._lib.flexar_group_allreduce_fp8(self._comms, self.nranks, ins, ous, tensors[0].numel(),
                                                      nv.dtype_code(tensors[0].dtype), nv.op_code(op),
                                                      _stream_handle(stream), wd, amx), "group_allreduce_fp8")
        return outs

    def collective(self, coll: str, ins: Sequence, outs: Sequence, op="sum", algo: Optional[str] = None, stream=None):
        """``coll`` = "reduce_scatter", "all_gather" or "all_to_all" for every rank of the group in one launch."""
        code = nv.COLLS[coll]
        count = outs[0].numel() if coll == "reduce_scatter" else (
            ins[0].numel() // self.nranks if coll == "all_to_all" else ins[0].numel())
        a = (ctypes.c_void_p * self.nranks)(*[t.data_ptr() for t in ins])
        b = (ctypes.c_void_p * self.nranks)(*[t.data_ptr() for t in outs])
        nv.check(self._lib.flexar_group_collective(self._comms, self.nranks, code, a, b, count,
                                                   nv.dtype_code(ins[0].dtype), nv.op_code(op), _stream_handle(stream),
                                                   algo.encode() if algo else None), coll)
        return outs

    def broadcast(self, ins: Sequence, outs: Sequence, root: int = 0, algo: Optional[str] = None, stream=None):
        """Broadcast ``ins[root]`` into every ``outs[r]`` in one launch."""
        a = (ctypes.c_void_p * self.nranks)(*[t.data_ptr() for t in ins])
        b = (ctypes.c_void_p * self.nranks)(*[t.data_ptr() for t in outs])
        nv.check(self._lib.flexar_group_broadcast(self._comms, self.nranks, int(root), a, b, outs[0].numel(),
                                                  nv.dtype_code(outs[0].dtype), _stream_handle(stream),
                                                  algo.encode() if algo else None), "broadcast")
        return outs

    def check(self):
        for r in range(self.nranks):
            nv.check(self._lib.flexar_comm_check(self._comms[r]), f"rank {r}")

    def clear_error(self):
        for r in range(self.nranks):
            nv.check(self._lib.flexar_comm_clear_error(self._comms[r]), f"rank {r}")

    def close(self):
        if getattr(self, "_comms", None) is not None:
            for r in range(self.nranks):
                if self._comms[r]:
                    self._lib.flexar_comm_destroy(self._comms[r])
                    self._comms[r] = None
            self._comms = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
