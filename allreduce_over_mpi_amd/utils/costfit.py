"""Fit the runtime cost model to measurements.

The reference scores topologies with hand-set constants (cost_model/CostModel.h:1-119: lo, co, bo, o) and
never checks them against a run. flexar's selector (csrc/include/flexar/cost_model.hpp XgmiModel) is linear
in theta = (alpha_launch_us, alpha_sync_us, 1/link_gbps, 1/hbm_gbps) for every executor schedule:

    cost_us(spec, N, bytes) = f(spec, N, bytes) . theta        (f from flexar_model_features)

so the tuner's (spec, bytes, us) rows determine theta by least squares. The fit minimises the RELATIVE
error (rows weighted by 1 / measured us: a 4 KiB call and a 1 GiB call count alike) under theta >= 0
(scipy nnls), and returns the FLEXAR_MODEL string the runtime reads, the per-row predictions and the
argmin agreement with the measured winners.

    rows = [{"spec": "flat+pull", "bytes": 4194304, "us": 35.6}, ...]   # tools/flexar_tune.py --jsonl
    fit = fit_model(rows, nranks=8)
    os.environ["FLEXAR_MODEL"] = fit["FLEXAR_MODEL"]        # or Communicator.calibrate(rows)
"""
from __future__ import annotations

import math
from collections import defaultdict

from .. import _native as nv


HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak: no schedule streams HBM faster (csrc/include/flexar/calibration.hpp)


def fit_model(rows, nranks: int, links: int = 0, min_bytes: float = 0.0):
    """Least-squares fit of theta to measured rows ({"spec", "bytes", "us"}). Returns a dict with the
    parameters, the FLEXAR_MODEL string, the rows' relative errors and the winner agreement."""
    import numpy as np
    from scipy.optimize import nnls

    feats, meas, used = [], [], []
    for r in rows:
        if r["bytes"] < min_bytes or not r.get("us") or r["us"] <= 0:
            continue
        f = nv.model_features(r["spec"], nranks, float(r["bytes"]), links, int(r.get("esize", 4)))
        if f is None:  # copy engines / LL above its cap: not in the linear model
            continue
        feats.append(f)
        meas.append(float(r["us"]))
        used.append(r)
    if len(used) < 4:
        raise ValueError("need at least 4 measurements of executor schedules to fit 4 parameters")
    A = np.asarray(feats, dtype=np.float64)
    y = np.asarray(meas, dtype=np.float64)
    w = 1.0 / y  # relative error
    # column scaling keeps nnls well conditioned (features span microseconds to gigabytes)
    colscale = np.maximum(np.abs(A * w[:, None]).max(axis=0), 1e-30)
    # theta >= lb: the HBM term is bounded by the part's peak, as in the native fit (calibration.hpp
    # kHbmPeakGBps); theta = lb + phi, phi >= 0
    lb = np.array([0.0, 0.0, 0.0, 1.0 / HBM_PEAK_GBPS])
    phi_s, _ = nnls(A * w[:, None] / colscale, y * w - (A * w[:, None]) @ lb)
    theta = lb + phi_s / colscale
    alpha_launch, alpha_sync, inv_link, inv_hbm = (float(v) for v in theta)
    # a parameter the data never exercised (zero column) or fitted to 0 keeps a finite bandwidth
    link_gbps = 1.0 / inv_link if inv_link > 1e-12 else 1e6
    hbm_gbps = 1.0 / inv_hbm if inv_hbm > 1e-12 else 1e6
    pred = A @ theta
    rel = np.abs(pred - y) / y
    # winner agreement per size, full specs: the measured winner must be the model's argmin among the
    # measured specs (flat+pull and flat+zc+push are different programs with different costs). Protocol
    # variants of one program ("+wt", "+nts") have identical features: the model ranks them as a tie, and
    # the winner counts as picked when it is tied for the model's minimum. `regret` = measured time of the
    # model's pick over the measured best - 1 (what following the model costs at that size).
    by_size = defaultdict(list)
    for r, p in zip(used, pred):
        by_size[r["bytes"]].append((r["us"], p, r["spec"]))
    agree, sizes, regrets = 0, [], []
    for b, cands in sorted(by_size.items()):
        meas_best, _, best_meas = min(cands)
        pmin = min(c[1] for c in cands)
        pick = min(cands, key=lambda c: (c[1], c[0]))  # the model's argmin (ties: its fastest member)
        ok = any(c[2] == best_meas and c[1] <= pmin * (1 + 1e-9) for c in cands)
        regret = pick[0] / meas_best - 1.0
        agree += ok
        regrets.append(regret)
        sizes.append({"bytes": b, "measured_winner": best_meas, "model_winner": pick[2], "agree": ok,
                      "regret": round(regret, 4)})
    return {
        "alpha_launch_us": alpha_launch, "alpha_sync_us": alpha_sync, "link_gbps": link_gbps,
        "hbm_gbps": hbm_gbps, "links": links,
        "FLEXAR_MODEL": f"{alpha_launch:.4g},{alpha_sync:.4g},{link_gbps:.6g},{hbm_gbps:.6g}"
                        + (f",{links}" if links > 0 else ""),
        "median_rel_err": float(np.median(rel)), "max_rel_err": float(rel.max()), "rows": len(used),
        "winner_agreement": agree / max(1, len(by_size)), "sizes": sizes,
        "max_regret": float(max(regrets)) if regrets else 0.0,
    }


def synthetic_rows(theta, nranks: int, specs, sizes, links: int = 0, noise: float = 0.0, seed: int = 0):
    """Rows generated from known theta (alpha_launch, alpha_sync, link_gbps, hbm_gbps) - for tests."""
    import random

    rnd = random.Random(seed)
    a, b, link, hbm = theta
    out = []
    for spec in specs:
        for s in sizes:
            f = nv.model_features(spec, nranks, float(s), links)
            if f is None:
                continue
            us = f[0] * a + f[1] * b + f[2] / link + f[3] / hbm
            if noise:
                us *= math.exp(rnd.gauss(0.0, noise))
            out.append({"spec": spec, "bytes": s, "us": us})
    return out
