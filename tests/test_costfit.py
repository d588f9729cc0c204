"""Cost-model calibration (allreduce_over_mpi_amd/utils/costfit.py, XgmiModel::features).

* features reproduce the model: f . theta == flexar_model_cost_us for every executor schedule;
* a fit on synthetic timings generated from known parameters recovers them;
* on the round-1 shared-GPU tuner measurements (profiles/r1_rehearsal/tune_shared4.jsonl) the fitted
  model picks the measured winner's schedule family at most sizes, where the default constants do not.
"""
import json
import os

import pytest

from allreduce_over_mpi_amd import _native as nv
from allreduce_over_mpi_amd.utils.costfit import fit_model, synthetic_rows

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPECS8 = ["oneshot", "ll", "flat+pull", "flat+push", "ring", "ring:2", "ring:4", "rhd+pull", "tree:2,4+pull",
          "tree:4,2+pull"]
SIZES = [4 << 10, 64 << 10, 1 << 20, 16 << 20, 256 << 20]


def test_features_reproduce_model_cost(monkeypatch):
    monkeypatch.setenv("FLEXAR_MODEL", "5,3,70,4500,7")
    for spec in SPECS8:
        for b in SIZES:
            f = nv.model_features(spec, 8, b)
            if f is None:
                assert spec == "ll" and b > (1 << 20)
                continue
            want = nv.model_cost_us(spec, 8, b)
            got = f[0] * 5 + f[1] * 3 + f[2] / 70 + f[3] / 4500
            assert abs(got - want) <= 1e-9 * max(1.0, want), (spec, b, got, want)
    assert nv.model_features("dma", 8, 1 << 20) is None  # copy engines: separate terms


@pytest.mark.parametrize("noise", [0.0, 0.02])
def test_fit_recovers_known_parameters(noise):
    theta = (7.5, 3.2, 48.0, 5200.0)
    rows = synthetic_rows(theta, 8, SPECS8, SIZES + [256 << 10, 4 << 20, 64 << 20], links=7, noise=noise)
    fit = fit_model(rows, 8, links=7)
    tol = 1e-6 if noise == 0 else 0.1
    for k, v in zip(("alpha_launch_us", "alpha_sync_us", "link_gbps", "hbm_gbps"), theta):
        assert abs(fit[k] - v) <= tol * v, (k, fit[k], v)
    assert fit["median_rel_err"] <= (1e-9 if noise == 0 else 0.05)
    assert fit["winner_agreement"] >= (1.0 if noise == 0 else 0.6)
    assert fit["FLEXAR_MODEL"].count(",") == 4


def test_fit_on_round1_shared_gpu_measurements():
    path = os.path.join(REPO, "profiles", "r1_rehearsal", "tune_shared4.jsonl")
    rows = [json.loads(line) for line in open(path) if line.strip()]
    fit = fit_model(rows, 4, links=1)  # ranks sharing one GPU: one "link", the shared HBM
    # bandwidth-bound sizes (>= 1 MiB): the fitted model picks the measured winner's schedule family.
    # Below that, 4 processes time-slice one GPU: ll vs oneshot differ by a few us out of 28-45 us
    # (launch-bound, alpha_launch fits ~39 us) and the measured order flips between neighbouring sizes.
    assert all(s["agree"] for s in fit["sizes"] if s["bytes"] >= 1 << 20), fit["sizes"]
    assert fit["winner_agreement"] >= 4 / 7, fit["sizes"]
    assert fit["median_rel_err"] < 0.25
    # ... where the uncalibrated defaults do worse (they predate any measurement)
    default_pick = 0
    for s in fit["sizes"]:
        cands = [r for r in rows if r["bytes"] == s["bytes"] and nv.model_features(r["spec"], 4, r["bytes"]) is not None]
        best = min(cands, key=lambda r: nv.model_cost_us(r["spec"], 4, r["bytes"]))["spec"]
        default_pick += best.split("+")[0] == s["measured_winner"].split("+")[0]
    assert fit["winner_agreement"] * len(fit["sizes"]) >= default_pick


def test_fit_needs_enough_rows():
    with pytest.raises(ValueError):
        fit_model([{"spec": "flat", "bytes": 4096, "us": 10.0}], 8)
