"""Connect-time calibration and probe agreement, host side.

* the native fit (csrc/include/flexar/calibration.hpp fit_theta: non-negative least squares on relative
  errors by support enumeration) recovers known constants from synthetic timings and agrees with the
  scipy fit of utils/costfit.py;
* the on-disk cache round-trips theta bit-exactly, a key mismatch (another node shape, world size, link
  count, disabled family or library version) is a miss, and a corrupt file is a miss;
* probe agreement (readiness.hpp probe_agree): the minimum link count is installed everywhere; asymmetric
  link classes or different settings fail with a message naming the ranks.
The device half - timing calib_points() on the links, max over ranks, install - is
tests/test_gpu_calibration.py.
"""
import ctypes
import struct

import pytest

from allreduce_over_mpi_amd import _native as nv
from allreduce_over_mpi_amd.utils.costfit import fit_model, synthetic_rows

MiB = 1 << 20


def _synthetic(theta, n, links, noise=0.0, seed=0):
    pts = nv.calib_points(n)
    specs = sorted({p[0] for p in pts})
    sizes = sorted({p[1] for p in pts})
    return synthetic_rows(theta, n, specs, sizes, links=links, noise=noise, seed=seed)


@pytest.mark.parametrize("n,links", [(2, 1), (4, 1), (8, 7), (8, 1)])
def test_native_fit_recovers_known_constants(n, links):
    theta = (9.0, 3.5, 55.0, 4800.0)
    rows = _synthetic(theta, n, links)
    fit = nv.calib_fit(rows, n, links)
    for k, v in zip(("alpha_launch_us", "alpha_sync_us", "link_gbps", "hbm_gbps"), theta):
        assert fit[k] == pytest.approx(v, rel=1e-6), (k, fit)
    assert fit["median_rel_err"] < 1e-9 and fit["rows"] == len(rows)


def test_native_fit_matches_scipy_on_noisy_rows():
    theta = (7.5, 4.2, 48.0, 5200.0)
    rows = _synthetic(theta, 8, 7, noise=0.03, seed=3)
    a = nv.calib_fit(rows, 8, 7)
    b = fit_model(rows, 8, links=7)
    for k in ("alpha_launch_us", "alpha_sync_us", "link_gbps", "hbm_gbps"):
        assert a[k] == pytest.approx(b[k], rel=1e-3), (k, a, b)


def test_calibration_points_identify_every_constant():
    """The measurement set must separate the four constants: its feature matrix has full rank."""
    import numpy as np

    for n, links in ((2, 1), (4, 1), (8, 7)):
        f = np.array([nv.model_features(s, n, b, links) for s, b in nv.calib_points(n)])
        assert np.linalg.matrix_rank(f / np.abs(f).max(axis=0)) == 4, (n, f)


def test_fit_keeps_constants_non_negative():
    # pure bandwidth rows with a negative intercept in an unconstrained fit: alpha must clamp at 0
    rows = [{"spec": "flat+pull", "bytes": b, "us": b / 4e5 - 0.5} for b in (4 * MiB, 16 * MiB, 64 * MiB, 256 * MiB)]
    rows += [{"spec": "ring", "bytes": b, "us": b / 2e5} for b in (4 * MiB, 64 * MiB)]
    fit = nv.calib_fit(rows, 4, 1)
    assert fit["alpha_launch_us"] >= 0 and fit["alpha_sync_us"] >= 0


def test_cache_round_trip_and_key_mismatch(tmp_path, monkeypatch):
    monkeypatch.setenv("FLEXAR_CALIB_DIR", str(tmp_path / "calib"))
    key = nv.calib_key("gfx950", 8, 7, "x7m0s0p0u0o0", 0)
    path = nv.calib_path(key)
    assert path.startswith(str(tmp_path / "calib"))
    assert nv.calib_load(path, key) is None  # nothing cached yet
    theta = [6.123456789012345, 3.25, 1 / 61.7, 1 / 5123.4]
    nv.calib_store(path, key, theta, [{"spec": "flat+pull", "bytes": 4 * MiB, "us": 35.5}])
    assert nv.calib_load(path, key) == theta  # bit-exact (%.17g)
    # every input of the key changes it (and the file name)
    others = [nv.calib_key("gfx942", 8, 7, "x7m0s0p0u0o0", 0), nv.calib_key("gfx950", 4, 7, "x7m0s0p0u0o0", 0),
              nv.calib_key("gfx950", 8, 1, "x7m0s0p0u0o0", 0), nv.calib_key("gfx950", 8, 7, "x0m0s7p0u0o0", 0),
              nv.calib_key("gfx950", 8, 7, "x7m0s0p0u0o0", 2)]
    assert len({key, *others}) == 6
    for k in others:
        assert nv.calib_path(k) != path
        assert nv.calib_load(path, k) is None  # the file's key line must match exactly
    assert "flexar=" + nv.lib().flexar_version().decode() in key


def test_corrupt_cache_is_a_miss(tmp_path):
    key = nv.calib_key("gfx950", 2, 1, "x0m0s1p0u0o0", 0)
    p = tmp_path / "c.txt"
    p.write_text(key + "\n1.0 nan 2 3\n")
    assert nv.calib_load(str(p), key) is None
    p.write_text(key + "\n1.0 -2 2 3\n")
    assert nv.calib_load(str(p), key) is None
    p.write_text(key + "\n")
    assert nv.calib_load(str(p), key) is None


def _blob(rank, links, cls, fp=1234, fixed=0, magic=0xF1E8B10B, resident=0):
    c = list(cls) + [0] * (16 - len(cls))
    return struct.pack("<IiiiQ16b16bii", magic, rank, links, fixed, fp, *c, *([1] * 16), resident, 0)


def _agree(blobs):
    assert len(blobs[0]) == nv.lib().flexar_probe_blob_size()
    out = ctypes.c_int(0)
    rc = nv.lib().flexar_probe_agree(b"".join(blobs), len(blobs), ctypes.byref(out))
    return (out.value, None) if rc == 0 else (None, nv.last_error())


XGMI, SAME, PCIE, UNK = 2, 1, 3, 0


def test_probe_agreement_takes_the_minimum_links():
    n = 4
    cls = lambda r: [SAME if p == r else XGMI for p in range(n)]  # noqa: E731
    links, err = _agree([_blob(r, 3 if r != 2 else 1, cls(r)) for r in range(n)])
    assert err is None and links == 1
    links, err = _agree([_blob(r, 3, cls(r)) for r in range(n)])
    assert links == 3


def test_probe_agreement_rejects_asymmetric_link_classes():
    n = 4
    views = [[SAME if p == r else XGMI for p in range(n)] for r in range(n)]
    views[2] = [SAME if p == 2 else PCIE for p in range(n)]  # rank 2 sees everyone over PCIe
    links, err = _agree([_blob(r, 3, views[r]) for r in range(n)])
    assert links is None and "disagree on the machine shape" in err and "rank 2" in err and "pcie" in err


def test_probe_agreement_tolerates_invisible_peers():
    n = 3
    views = [[SAME, UNK, XGMI], [UNK, SAME, UNK], [XGMI, UNK, SAME]]  # rank 1 sees nobody (HIP_VISIBLE_DEVICES)
    links, err = _agree([_blob(r, 2, views[r]) for r in range(n)])
    assert err is None and links == 2


def test_probe_agreement_rejects_different_settings():
    n = 2
    views = [[SAME, XGMI], [XGMI, SAME]]
    _, err = _agree([_blob(0, 1, views[0], fp=1), _blob(1, 1, views[1], fp=2)])
    assert err and "different settings" in err
    _, err = _agree([_blob(0, 1, views[0], fixed=7), _blob(1, 1, views[1], fixed=0)])
    assert err and "different settings" in err
    _, err = _agree([_blob(0, 1, views[0]), _blob(1, 1, views[1], magic=1)])
    assert err and "malformed" in err


@pytest.mark.parametrize("n,links", [(4, 1), (8, 7)])
def test_fit_bounds_the_hbm_term_by_the_peak(n, links):
    """Rows generated with an unphysical HBM rate (20 TB/s, what an unidentified link/HBM split can produce
    on ranks sharing one device): both fits keep hbm_gbps at or below the part's 8 TB/s peak and agree."""
    rows = _synthetic((9.0, 3.5, 55.0, 20000.0), n, links)
    a = nv.calib_fit(rows, n, links)
    b = fit_model(rows, n, links=links)
    assert a["hbm_gbps"] <= 8000.0 * (1 + 1e-9), a
    assert b["hbm_gbps"] <= 8000.0 * (1 + 1e-9), b
    for k in ("alpha_launch_us", "alpha_sync_us", "link_gbps", "hbm_gbps"):
        assert a[k] == pytest.approx(b[k], rel=1e-3), (k, a, b)


def test_probe_agreement_installs_the_minimum_resident_grid():
    """the executor grid is clamped to the resident workgroups; every rank must clamp alike, so the
    minimum over the ranks that know their count is agreed on (0 = unknown, ignored)."""
    n = 3
    cls = lambda r: [SAME if p == r else XGMI for p in range(n)]  # noqa: E731
    links, resident = ctypes.c_int(0), ctypes.c_int(-1)
    blobs = b"".join(_blob(r, 2, cls(r), resident=res) for r, res in enumerate((1024, 768, 0)))
    assert nv.lib().flexar_probe_agree_resident(blobs, n, ctypes.byref(links), ctypes.byref(resident)) == 0
    assert (links.value, resident.value) == (2, 768)
    blobs = b"".join(_blob(r, 2, cls(r)) for r in range(n))
    assert nv.lib().flexar_probe_agree_resident(blobs, n, ctypes.byref(links), ctypes.byref(resident)) == 0
    assert resident.value == 0


def test_calib_mode_does_not_change_the_cache_key(monkeypatch):
    """FLEXAR_CALIB=force writes the cache that default runs read; unset and "1" are one mode."""
    keys = {}
    for v in (None, "1", "force", "0"):
        if v is None:
            monkeypatch.delenv("FLEXAR_CALIB", raising=False)
        else:
            monkeypatch.setenv("FLEXAR_CALIB", v)
        keys[v] = (nv.lib().flexar_settings_fingerprint(0), nv.lib().flexar_settings_fingerprint(1))
    assert len({k[0] for k in keys.values()}) == 1  # cache-key form: no calibration mode in it
    assert keys[None][1] == keys["1"][1] != keys["force"][1] != keys["0"][1]  # connect form: normalised mode

