"""ctypes binding of ``libflexar.so`` (the native runtime; see csrc/include/flexar/flexar.h).

The library is loaded from the package's in-tree ``_lib/`` directory (built by
``_build.build()``), never from site-packages, so the GPU box loads exactly the
code object compiled here. ``import torch`` happens first so the HIP runtime
already mapped by torch (same soname ``libamdhip64.so.7``) is the one the
library binds to — one HIP runtime per process.
"""
from __future__ import annotations

import ctypes
import os
import threading

from . import _build

_lock = threading.Lock()
_lib = None

DTYPES = {
    "float32": 0, "float16": 1, "bfloat16": 2, "float64": 3, "fp8_e4m3": 4, "fp8_e5m2": 5,
    "int8": 6, "uint8": 7, "int16": 8, "uint16": 9, "int32": 10, "uint32": 11, "int64": 12,
    "uint64": 13, "bool": 14,
}
OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4, "band": 5, "bor": 6, "bxor": 7}
ERRORS = {0: "ok", 1: "invalid", 2: "unsupported", 3: "hip", 4: "timeout", 5: "state", 6: "nomem", 7: "rccl"}


class FlexarError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(f"flexar error {rc} ({ERRORS.get(rc, '?')}): {msg}")
        self.rc = rc


# int (*agree)(void* ctx) of flexar_comm_destroy_agreed
AGREE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)


def _sig(lib):
    c = ctypes
    vp, sz, i, f, d, cp = c.c_void_p, c.c_size_t, c.c_int, c.c_float, c.c_double, c.c_char_p
    u64, u32 = c.c_uint64, c.c_uint32
    table = {
        "flexar_version": (cp, []),
        "flexar_last_error": (cp, []),
        "flexar_dtype_size": (sz, [i]),
        "flexar_comm_create": (i, [i, i, i, sz, c.POINTER(vp)]),
        "flexar_handle_size": (sz, []),
        "flexar_comm_export": (i, [vp, vp]),
        "flexar_comm_connect": (i, [vp, vp]),
        "flexar_comm_destroy": (i, [vp]),
        "flexar_comm_destroy_local": (i, [vp]),
        "flexar_comm_destroy_agreed": (i, [vp, AGREE_FN, vp]),
        "flexar_comm_last_spec": (i, [vp, cp, sz]),
        "flexar_parked_bytes": (u64, []),
        "flexar_comm_set_zc_auto": (i, [vp, i]),
        "flexar_comm_resync": (i, [vp]),
        "flexar_comm_host_agree": (i, [vp, c.c_uint64, i, c.POINTER(c.c_uint64)]),
        "flexar_comm_host_page_check": (i, [vp, c.POINTER(i)]),
        "flexar_comm_host_page_drop": (i, [vp]),
        "flexar_host_barrier_run": (i, [cp, i, i, i, c.c_uint64, i]),
        "flexar_host_page_open": (vp, [cp, i, i, u64]),
        "flexar_host_page_shared": (i, [vp, u64, c.POINTER(i)]),
        "flexar_host_page_close": (None, [vp]),
        "flexar_comm_selftest_note": (i, [vp, cp, sz]),
        "flexar_comm_rank": (i, [vp]),
        "flexar_comm_size": (i, [vp]),
        "flexar_comm_set_algo": (i, [vp, cp]),
        "flexar_comm_set_grid": (i, [vp, i, i]),
        "flexar_comm_set_xfer_chunk": (i, [vp, u64]),
        "flexar_comm_set_tune_table": (i, [vp, cp]),
        "flexar_allreduce": (i, [vp, vp, vp, sz, i, i, vp]),
        "flexar_allreduce_ex": (i, [vp, vp, vp, sz, i, i, vp, cp, f]),
        "flexar_comm_check": (i, [vp]),
        "flexar_comm_clear_error": (i, [vp]),
        "flexar_comm_describe": (i, [vp, sz, i, cp, sz]),
        "flexar_comm_stats": (i, [vp, cp, sz]),
        "flexar_group_create": (i, [i, i, sz, c.POINTER(vp)]),
        "flexar_group_allreduce": (i, [c.POINTER(vp), i, c.POINTER(vp), c.POINTER(vp), sz, i, i, vp, cp, f]),
        "flexar_reduce": (i, [vp, c.POINTER(vp), i, sz, i, i, f, vp]),
        "flexar_reduce_host": (i, [vp, c.POINTER(vp), i, sz, i, i, f]),
        "flexar_parse_ft_topo": (i, [cp, i, cp, sz]),
        "flexar_count_factorizations": (u64, [i]),
        "flexar_ring_order": (i, [i, i, i, vp]),
        "flexar_enumerate_plans": (i, [i, cp, sz]),
        "flexar_model_cost_us": (d, [cp, i, d]),
        "flexar_select_plan": (i, [i, d, cp, sz]),
        "flexar_legacy_cost": (d, [cp, i, d]),
        "flexar_plan_dump": (i, [cp, i, i, sz, i, cp, sz]),
        "flexar_simulate": (i, [cp, i, sz, i, i, c.POINTER(vp), c.POINTER(vp), i, i, i, f]),
        "flexar_simulate_coll": (i, [i, cp, i, sz, i, i, c.POINTER(vp), c.POINTER(vp), i, i, f]),
        "flexar_reduce_scatter": (i, [vp, vp, vp, sz, i, i, vp, cp]),
        "flexar_all_gather": (i, [vp, vp, vp, sz, i, vp, cp]),
        "flexar_group_collective": (i, [c.POINTER(vp), i, i, c.POINTER(vp), c.POINTER(vp), sz, i, i, vp, cp]),
        "flexar_broadcast": (i, [vp, vp, vp, sz, i, i, vp, cp]),
        "flexar_all_to_all": (i, [vp, vp, vp, sz, i, vp]),
        "flexar_all_to_all_ex": (i, [vp, vp, vp, sz, i, vp, cp]),
        "flexar_amax": (i, [vp, sz, i, vp, vp]),
        "flexar_quantize_fp8": (i, [vp, i, vp, sz, vp, f, vp]),
        "flexar_dequantize_fp8": (i, [vp, vp, i, sz, vp, f, vp]),
        "flexar_mx_pack": (i, [vp, i, vp, sz, i, vp]),
        "flexar_mx_unpack_sum": (i, [vp, sz, i, sz, i, vp, vp]),
        "flexar_mx_unpack_sum_scaled": (i, [vp, sz, i, sz, i, f, vp, vp]),
        "flexar_group_broadcast": (i, [c.POINTER(vp), i, i, c.POINTER(vp), c.POINTER(vp), sz, i, vp, cp]),
        "flexar_simulate_bcast": (i, [cp, i, sz, i, i, c.POINTER(vp), c.POINTER(vp), i, i]),
        "flexar_simulate_typed": (i, [cp, i, sz, i, i, c.POINTER(vp), c.POINTER(vp), i, i, f, f]),
        "flexar_simulate_msg": (i, [cp, i, sz, i, i, c.POINTER(vp), c.POINTER(vp), i, f]),
        "flexar_msg_plan_dump": (i, [cp, i, i, sz, i, cp, sz]),
        "flexar_allreduce_fp8": (i, [vp, vp, vp, sz, i, i, vp, i, vp, cp]),
        "flexar_group_allreduce_fp8": (i, [c.POINTER(vp), i, c.POINTER(vp), c.POINTER(vp), sz, i, i, vp, i,
                                            c.POINTER(vp)]),
        "flexar_comm_selftest": (i, [vp, u32, c.POINTER(u32)]),
        "flexar_comm_set_disabled": (i, [vp, u32]),
        "flexar_comm_disabled": (u32, [vp]),
        "flexar_comm_topology": (i, [vp, cp, sz]),
        "flexar_comm_predict_us": (d, [vp, cp, d]),
        "flexar_comm_set_model": (i, [vp, d, d, d, d, i]),
        "flexar_rccl_available": (i, []),
        "flexar_rccl_unique_id": (i, [vp, sz]),
        "flexar_comm_init_msg": (i, [vp, vp]),
        "flexar_comm_connect_msg_only": (i, [vp]),
        "flexar_reg_handle_size": (sz, []),
        "flexar_reg_export": (i, [vp, vp, sz, vp]),
        "flexar_reg_open": (i, [vp, vp, sz, vp, c.POINTER(i)]),
        "flexar_reg_close": (i, [vp, i]),
        "flexar_reg_count": (i, [vp]),
        "flexar_reg_find": (i, [vp, vp, sz]),
        "flexar_reg_ids": (i, [vp, c.POINTER(i), i]),
        "flexar_zc_decide": (i, [cp, i, d, i, u32, c.POINTER(i), cp, sz]),
        "flexar_model_features": (i, [cp, i, d, i, c.POINTER(d)]),
        "flexar_model_features_ex": (i, [cp, i, d, i, i, c.POINTER(d)]),
        "flexar_program_cost": (i, [cp, i, i, sz, i, i, c.POINTER(d)]),
        "flexar_select_plan_ex": (i, [i, d, i, i, i, cp, sz]),
        "flexar_apply_partials": (i, [cp, i, d, i, i, cp, sz]),
        "flexar_kernel_info": (i, [i, i, i, i, c.POINTER(i), c.POINTER(i)]),
        "flexar_kernel_info_ex": (i, [i, i, i, i, c.POINTER(i), c.POINTER(i), c.POINTER(i)]),
        "flexar_downgrade_spec": (i, [cp, i, u32, i, cp, sz]),
        "flexar_direct_links": (i, [c.POINTER(c.c_int32), c.POINTER(c.c_int32), i, i]),
        "flexar_probe_blob_size": (sz, []),
        "flexar_probe_agree": (i, [vp, i, c.POINTER(i)]),
        "flexar_probe_agree_resident": (i, [vp, i, c.POINTER(i), c.POINTER(i)]),
        "flexar_settings_fingerprint": (c.c_uint64, [i]),
        "flexar_comm_probe_export": (i, [vp, vp]),
        "flexar_comm_probe_agree": (i, [vp, vp]),
        "flexar_comm_calibrate": (i, [vp, i, cp, sz]),
        "flexar_comm_calibration": (i, [vp, cp, sz]),
        "flexar_comm_reset_model": (i, [vp]),
        "flexar_comm_model_hash": (u64, [vp]),
        "flexar_calib_fit": (i, [i, cp, c.POINTER(d), c.POINTER(d), i, i, i, c.POINTER(d)]),
        "flexar_calib_key": (i, [cp, i, i, cp, u32, cp, sz]),
        "flexar_calib_path": (i, [cp, cp, sz]),
        "flexar_calib_load": (i, [cp, cp, c.POINTER(d)]),
        "flexar_calib_store": (i, [cp, cp, c.POINTER(d), i, cp, c.POINTER(d), c.POINTER(d)]),
        "flexar_calib_points": (i, [i, cp, sz]),
        "flexar_crash_report_install": (None, []),
        "flexar_crash_report_dump": (None, [cp]),
        "flexar_crumb": (None, [cp, cp, i, i, u64, u64]),
        "flexar_test_fatal": (None, [i]),
    }
    for name, (res, args) in table.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib():
    """Load (building first if needed) the native library."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            try:
                import torch  # noqa: F401  (bind to torch's HIP runtime first)
            except Exception:
                pass
            path = _build.LIB_PATH
            if os.environ.get("FLEXAR_LIB_PATH"):  # A/B experiments: another build of the library
                path = os.environ["FLEXAR_LIB_PATH"]
            elif _build.needs_build() and os.environ.get("FLEXAR_NO_BUILD") != "1":
                path = _build.build()
            if not os.path.exists(path):
                raise FlexarError(5, f"native library missing: {path} (run __graft_entry__.build())")
            l = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
            _sig(l)
            _load_fastcall(l)
            # fatal-signal / std::terminate report of the last flexar launches (crumbs.hpp); chains to the
            # handlers installed before (Python's faulthandler under pytest); FLEXAR_CRASH_REPORT=0: off
            l.flexar_crash_report_install()
            _lib = l
    return _lib


# Fast-call path (csrc/python/fastcall.c): the per-step collectives bypass ctypes' argument conversion.
# FAST is the module (None if it was not built) and AR/RS/AG the C entry points' addresses.
FAST = None
AR = RS = AG = 0


def _load_fastcall(l):
    global FAST, AR, RS, AG
    import importlib.machinery
    import importlib.util

    p = _build.FASTCALL_PATH
    if not os.path.exists(p):
        return
    loader = importlib.machinery.ExtensionFileLoader("_fastcall", p)
    spec = importlib.util.spec_from_file_location("_fastcall", p, loader=loader)
    m = importlib.util.module_from_spec(spec)
    loader.exec_module(m)
    addr = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
    AR, RS, AG = addr(l.flexar_allreduce_ex), addr(l.flexar_reduce_scatter), addr(l.flexar_all_gather)
    FAST = m


def log_warn(msg: str):
    """A warning on stderr in the native logger's format (silenced by FLEXAR_LOG_LEVEL=error)."""
    if os.environ.get("FLEXAR_LOG_LEVEL", "warn").lower() not in ("error", "none", "off"):
        import sys

        print(f"[flexar W] {msg}", file=sys.stderr, flush=True)


def crumb(what: str, label: str = "", rank: int = -1, nranks: int = 0, epoch: int = 0, nbytes: int = 0):
    """A phase breadcrumb in the native ring (printed by the crash report)."""
    lib().flexar_crumb(what.encode(errors="replace"), label.encode(errors="replace"), int(rank), int(nranks),
                       int(epoch), int(nbytes))


_T0 = None


def phase(what: str, rank: int = -1, nranks: int = 0, echo: bool = None):
    """A start-up / section phase: a native breadcrumb, and (FLEXAR_PHASE_LOG=1, or echo=True) one stderr
    line from THIS rank with the wall-clock time (comparable with torch's log stamps) and the seconds since
    this process first logged a phase - so a failure on any rank names the phase that rank reached."""
    import time

    global _T0
    if _T0 is None:
        _T0 = time.monotonic()
    if _lib is not None:
        crumb("phase", what, rank, nranks)
    if echo is None:
        echo = os.environ.get("FLEXAR_PHASE_LOG") == "1"
    if echo:
        import sys

        now = time.time()
        stamp = time.strftime("%H:%M:%S", time.localtime(now)) + f".{int(now * 1000) % 1000:03d}"
        # one write(2) per line: ranks sharing a launcher's stderr must not split each other's lines
        sys.stderr.flush()
        os.write(2, f"[phase r{rank} {stamp} +{time.monotonic() - _T0:.3f}s] {what}\n".encode())


def last_error() -> str:
    return lib().flexar_last_error().decode(errors="replace")


def check(rc: int, what: str = ""):
    if rc != 0:
        raise FlexarError(rc, (what + ": " if what else "") + last_error())


def lib_path() -> str:
    return _build.LIB_PATH


def dtype_code(dtype) -> int:
    """Map a torch dtype / numpy dtype / name to the flexar dtype enum."""
    name = str(dtype).replace("torch.", "")
    alias = {"float": "float32", "half": "float16", "double": "float64", "float8_e4m3fn": "fp8_e4m3",
             "float8_e5m2": "fp8_e5m2", "int": "int32", "long": "int64", "uint8": "uint8"}
    name = alias.get(name, name)
    if name not in DTYPES:
        raise FlexarError(2, f"unsupported dtype {dtype}")
    return DTYPES[name]


def op_code(op) -> int:
    if isinstance(op, int):
        return op
    name = str(op).lower().replace("reduceop.", "").replace("redopttype.", "")
    alias = {"product": "prod", "average": "avg", "mean": "avg"}
    name = alias.get(name, name)
    if name not in OPS:
        raise FlexarError(2, f"unsupported reduce op {op}")
    return OPS[name]


def _strbuf(n=1 << 16):
    return ctypes.create_string_buffer(n)


def parse_ft_topo(ft_topo: str | None, nranks: int) -> str:
    b = _strbuf(256)
    check(lib().flexar_parse_ft_topo((ft_topo or "").encode(), nranks, b, 256), "parse_ft_topo")
    return b.value.decode()


def count_factorizations(n: int) -> int:
    return int(lib().flexar_count_factorizations(n))


def ring_order(nranks: int, channel: int, channels: int = 1) -> tuple[list[int], int]:
    """(rank order of ring ``channel`` of a ``channels``-channel ring, the most channels N ranks allow)."""
    buf = (ctypes.c_int * nranks)()
    m = lib().flexar_ring_order(nranks, channel, channels, buf)
    if m < 0:
        raise ValueError("bad ring_order arguments")
    return list(buf), int(m)


def enumerate_plans(nranks: int) -> list[str]:
    b = _strbuf(1 << 20)
    check(lib().flexar_enumerate_plans(nranks, b, 1 << 20), "enumerate_plans")
    return [x for x in b.value.decode().split("\n") if x]


def model_cost_us(spec: str, nranks: int, nbytes: float) -> float:
    v = lib().flexar_model_cost_us(spec.encode(), nranks, float(nbytes))
    if v < 0:
        raise FlexarError(1, last_error())
    return v


def model_features(spec: str, nranks: int, nbytes: float, links: int = 0, esize: int = 4):
    """Linear cost features of ``spec``: cost_us = f . (alpha_launch, alpha_sync, 1/link_gbps, 1/hbm_gbps),
    read off the compiled programs for elements of ``esize`` bytes; None for schedules outside the linear
    model (copy engines, LL above its size cap)."""
    out = (ctypes.c_double * 4)()
    rc = lib().flexar_model_features_ex(spec.encode(), nranks, float(nbytes), int(links), int(esize), out)
    if rc == 2:
        return None
    check(rc, "model_features")
    return list(out)


def program_cost(spec: str, rank: int, nranks: int, count: int, dtype="float32", links: int = 0) -> dict:
    """What rank's compiled program costs (csrc/include/flexar/cost_model.hpp program_cost): hand-offs,
    bytes over links (remote reads + writes), the busiest link's bytes phase by phase, HBM bytes."""
    out = (ctypes.c_double * 5)()
    check(lib().flexar_program_cost(spec.encode(), rank, nranks, int(count), dtype_code(dtype), int(links), out),
          "program_cost")
    return dict(zip(("handoffs", "link_bytes", "link_time_bytes", "hbm_read", "hbm_write"), list(out)))


def zc_decide(spec: str, nranks: int, nbytes: float, registered=True, named=False, auto=True, zc_auto=True,
              have_tune=False, disabled: int = 0):
    """The zero-copy policy on a concrete spec: (decision, spec) with decision 1 = switched to zero copy,
    -1 = fell back to staging, 0 = unchanged (csrc/include/flexar/zc_policy.hpp)."""
    flags = (1 if registered else 0) | (2 if named else 0) | (4 if auto else 0) | (8 if zc_auto else 0) | \
            (16 if have_tune else 0)
    dec = ctypes.c_int(0)
    b = _strbuf(256)
    check(lib().flexar_zc_decide(spec.encode(), nranks, float(nbytes), flags, disabled, ctypes.byref(dec), b, 256),
          "zc_decide")
    return dec.value, b.value.decode()


def select_plan(nranks: int, nbytes: float, dtype=None, op="sum", links: int = 0) -> str:
    """The cost model's choice for (nranks, nbytes); with ``dtype`` the typed form that call would run
    (FLEXAR_PARTIALS and FLEXAR_MODEL apply)."""
    b = _strbuf(256)
    if dtype is None and not links:
        check(lib().flexar_select_plan(nranks, float(nbytes), b, 256), "select_plan")
    else:
        check(lib().flexar_select_plan_ex(nranks, float(nbytes), dtype_code(dtype or "float32"), op_code(op),
                                          int(links), b, 256), "select_plan")
    return b.value.decode()


def apply_partials(spec: str, nranks: int, nbytes: float, dtype="bfloat16", op="sum") -> str:
    """The typed form ``spec`` runs for a call of ``dtype`` / ``op`` under FLEXAR_PARTIALS (cost_model.hpp)."""
    b = _strbuf(256)
    check(lib().flexar_apply_partials(spec.encode(), nranks, float(nbytes), dtype_code(dtype), op_code(op), b, 256),
          "apply_partials")
    return b.value.decode()


def _rows_args(rows):
    n = len(rows)
    specs = "\n".join(r["spec"] for r in rows).encode()
    b = (ctypes.c_double * max(1, n))(*[float(r["bytes"]) for r in rows])
    u = (ctypes.c_double * max(1, n))(*[float(r["us"]) for r in rows])
    return n, specs, b, u


def calib_fit(rows, nranks: int, links: int = 0, esize: int = 4) -> dict:
    """The native least-squares fit of the connect-time calibration (calibration.hpp fit_theta) on rows
    ({"spec", "bytes", "us"})."""
    out = (ctypes.c_double * 7)()
    n, specs, b, u = _rows_args(rows)
    check(lib().flexar_calib_fit(n, specs, b, u, nranks, int(links), int(esize), out), "calib_fit")
    keys = ("alpha_launch_us", "alpha_sync_us", "link_gbps", "hbm_gbps", "median_rel_err", "max_rel_err", "rows")
    return dict(zip(keys, list(out)))


def calib_key(arch: str, nranks: int, links: int, classes: str = "", disabled: int = 0) -> str:
    b = _strbuf(1024)
    check(lib().flexar_calib_key(arch.encode(), nranks, links, classes.encode(), disabled, b, 1024), "calib_key")
    return b.value.decode()


def calib_path(key: str) -> str:
    b = _strbuf(4096)
    check(lib().flexar_calib_path(key.encode(), b, 4096), "calib_path")
    return b.value.decode()


def calib_load(path: str, key: str):
    """theta (alpha_launch_us, alpha_sync_us, 1/link_gbps, 1/hbm_gbps) from the cache file, or None."""
    t = (ctypes.c_double * 4)()
    return list(t) if lib().flexar_calib_load(path.encode(), key.encode(), t) == 1 else None


def calib_store(path: str, key: str, theta, rows=()):
    t = (ctypes.c_double * 4)(*[float(x) for x in theta])
    n, specs, b, u = _rows_args(list(rows))
    check(lib().flexar_calib_store(path.encode(), key.encode(), t, n, specs, b, u), "calib_store")


def calib_points(nranks: int) -> list:
    b = _strbuf(4096)
    check(lib().flexar_calib_points(nranks, b, 4096), "calib_points")
    return [(ln.split()[0], int(ln.split()[1])) for ln in b.value.decode().splitlines() if ln.strip()]


def legacy_cost(widths, nranks: int, chunk: float) -> float:
    s = ",".join(str(w) for w in widths)
    return float(lib().flexar_legacy_cost(s.encode(), nranks, float(chunk)))


def plan_dump(spec: str, rank: int, nranks: int, count: int, dtype="float32") -> str:
    b = _strbuf(1 << 22)
    check(lib().flexar_plan_dump(spec.encode(), rank, nranks, count, dtype_code(dtype), b, 1 << 22), "plan_dump")
    return b.value.decode()


# protocol families (csrc/include/flexar/readiness.hpp)
FAMILIES = {"fence": 1, "wt": 2, "ll": 4, "dma": 8, "rccl": 16}


def family_names(mask: int) -> list[str]:
    return [k for k, v in FAMILIES.items() if mask & v]


def downgrade_spec(spec: str, nranks: int, disabled, allow_dma: bool = True) -> str:
    """The spec a call runs when the families in ``disabled`` (mask or names) failed the self-test."""
    if not isinstance(disabled, int):
        disabled = sum(FAMILIES[n] for n in disabled)
    b = _strbuf(256)
    check(lib().flexar_downgrade_spec(spec.encode(), nranks, disabled, int(allow_dma), b, 256), "downgrade_spec")
    return b.value.decode()


LINK_CLASSES = {"unknown": 0, "same-device": 1, "xgmi": 2, "pcie": 3, "other": 4}


def direct_links(classes, hops, self_rank: int) -> int:
    """Concurrent links the cost model assumes for probed per-peer link classes (names) and hop counts."""
    n = len(classes)
    a = (ctypes.c_int32 * n)(*[LINK_CLASSES[c] for c in classes])
    h = (ctypes.c_int32 * n)(*hops)
    return int(lib().flexar_direct_links(a, h, n, self_rank))


def kernel_info(dtype="float32", op="sum", kind: int = 0, proto: int = 0) -> dict:
    """Occupancy (512-thread workgroups per CU) and VGPRs of one kernel instantiation (needs a GPU).
    kind: 0 executor (proto 0 fence / 1 nts / 2 wt), 1 LL, 2 reduce, 3/4/5 typed executor (fp32 partials /
    e4m3 wire / e5m2 wire), 6/7 typed executor with the OCP MX e4m3 / e5m2 wire (the fan-in-8 class).
    ``scratch_bytes``: the private segment per lane (spills, stack objects)."""
    occ, regs, scr = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    check(lib().flexar_kernel_info_ex(dtype_code(dtype), op_code(op), kind, proto, ctypes.byref(occ), ctypes.byref(regs),
                                      ctypes.byref(scr)), "kernel_info")
    return {"blocks_per_cu": occ.value, "vgprs": regs.value, "scratch_bytes": scr.value}


def _ptr_array(ptrs):
    arr = (ctypes.c_void_p * len(ptrs))()
    for k, p in enumerate(ptrs):
        arr[k] = p
    return arr


def simulate(spec: str, inputs, op="sum", grid=2, ncalls=2, in_place=False, scale=1.0):
    """Run the device op programs on host numpy arrays (one thread per rank x block).

    ``inputs`` is a list of equally shaped contiguous numpy arrays (one per rank).
    Returns the list of per-rank outputs.
    """
    import numpy as np

    n = len(inputs)
    first = inputs[0]
    dt = {"float32": "float32", "float64": "float64", "int32": "int32", "int64": "int64", "int8": "int8",
          "uint8": "uint8", "int16": "int16", "uint16": "uint16", "uint32": "uint32",
          "uint64": "uint64", "bool": "bool"}.get(str(first.dtype))
    code = DTYPES[getattr(inputs, "flexar_dtype", None) or dt] if dt else None
    return _simulate_raw(spec, inputs, code, op, grid, ncalls, in_place, scale, np)


def _simulate_raw(spec, inputs, code, op, grid, ncalls, in_place, scale, np):
    n = len(inputs)
    ins = [np.ascontiguousarray(x) for x in inputs]
    outs = [np.empty_like(x) for x in ins]
    if in_place:
        for o, x in zip(outs, ins):
            o[...] = x
    rc = lib().flexar_simulate(spec.encode(), n, ins[0].size, code, op_code(op),
                               _ptr_array([x.ctypes.data for x in ins]),
                               _ptr_array([o.ctypes.data for o in outs]), grid, ncalls, int(in_place), float(scale))
    check(rc, "simulate")
    return outs


def simulate_typed(spec: str, inputs, dtype: str, op="sum", grid=2, ncalls=2, in_place=False, scale=1.0):
    """Like simulate() but with an explicit flexar dtype name for raw-bit arrays (bf16/fp16/fp8 as uint16/uint8)."""
    import numpy as np

    return _simulate_raw(spec, inputs, DTYPES[dtype], op, grid, ncalls, in_place, scale, np)


def simulate_mx(spec: str, inputs, dtype: str, op="sum", grid=2, ncalls=2, scale=1.0, pre=1.0):
    """Typed-staging programs ("+f32" / "+e4m3" / "+e5m2" suffix) on host arrays. ``inputs`` hold raw bits for
    16/8-bit dtypes (uint16 / uint8 arrays). ``pre`` is the fp8 pre-scale s (the device derives
    fp8_max / (N * amax))."""
    import numpy as np

    n = len(inputs)
    ins = [np.ascontiguousarray(x) for x in inputs]
    outs = [np.empty_like(x) for x in ins]
    rc = lib().flexar_simulate_typed(spec.encode(), n, ins[0].size, DTYPES[dtype], op_code(op),
                                     _ptr_array([x.ctypes.data for x in ins]), _ptr_array([o.ctypes.data for o in outs]),
                                     grid, ncalls, float(scale), float(pre))
    check(rc, "simulate_typed")
    return outs


def simulate_msg(spec: str, inputs, op="sum", ncalls=2, scale=1.0, dtype: str | None = None):
    """Run the message-transport plans (send/recv + local executor segments, what the RCCL transport posts)
    on host numpy arrays. Returns the per-rank outputs."""
    import numpy as np

    ins = [np.ascontiguousarray(x) for x in inputs]
    outs = [np.empty_like(x) for x in ins]
    code = DTYPES[dtype] if dtype else dtype_code(ins[0].dtype)
    check(lib().flexar_simulate_msg(spec.encode(), len(ins), ins[0].size, code, op_code(op),
                                    _ptr_array([x.ctypes.data for x in ins]), _ptr_array([o.ctypes.data for o in outs]),
                                    ncalls, float(scale)), "simulate_msg")
    return outs


def msg_plan(spec: str, rank: int, nranks: int, count: int, dtype="float32") -> dict:
    import json

    b = _strbuf(1 << 20)
    check(lib().flexar_msg_plan_dump(spec.encode(), rank, nranks, count, dtype_code(dtype), b, 1 << 20), "msg_plan")
    return json.loads(b.value.decode())


def reduce_host(srcs, op="sum", scale=1.0, dtype: str | None = None):
    import numpy as np

    srcs = [np.ascontiguousarray(s) for s in srcs]
    out = np.empty_like(srcs[0])
    code = DTYPES[dtype] if dtype else dtype_code(srcs[0].dtype)
    check(lib().flexar_reduce_host(out.ctypes.data, _ptr_array([s.ctypes.data for s in srcs]), len(srcs),
                                   srcs[0].size, code, op_code(op), float(scale)), "reduce_host")
    return out


COLLS = {"allreduce": 0, "reduce_scatter": 1, "all_gather": 2, "all_to_all": 4}


def simulate_coll(coll: str, spec: str, inputs, count: int, dtype: str = "float32", op="sum", grid=2, ncalls=2,
                  scale=1.0):
    """Simulate reduce_scatter (inputs N*count, outputs count), all_gather (inputs count, outputs N*count)
    or all_to_all (inputs and outputs N*count)."""
    import numpy as np

    n = len(inputs)
    ins = [np.ascontiguousarray(x) for x in inputs]
    out_n = count if coll == "reduce_scatter" else (n * count if coll in ("all_gather", "all_to_all") else count)
    outs = [np.zeros(out_n, dtype=ins[0].dtype) for _ in range(n)]
    rc = lib().flexar_simulate_coll(COLLS[coll], spec.encode(), n, count, DTYPES[dtype], op_code(op),
                                    _ptr_array([x.ctypes.data for x in ins]), _ptr_array([o.ctypes.data for o in outs]),
                                    grid, ncalls, float(scale))
    check(rc, "simulate_coll")
    return outs


def simulate_bcast(spec: str, data, nranks: int, root: int = 0, dtype: str = "float32", grid=2, ncalls=2):
    """Simulate a broadcast of the numpy array ``data`` (the root's input) to ``nranks`` ranks."""
    import numpy as np

    src = np.ascontiguousarray(data)
    ins = [src if r == root else np.zeros_like(src) for r in range(nranks)]
    outs = [np.zeros_like(src) for _ in range(nranks)]
    rc = lib().flexar_simulate_bcast(spec.encode(), nranks, src.size, DTYPES[dtype], root,
                                     _ptr_array([x.ctypes.data for x in ins]), _ptr_array([o.ctypes.data for o in outs]),
                                     grid, ncalls)
    check(rc, "simulate_bcast")
    return outs
