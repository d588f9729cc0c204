"""bench.py's wall-clock budget: optional items are dropped in a fixed order - the
calibration mini-sweep first, then config #4's tail sizes, then the grid sweep - decided on the agreed
(max over ranks) elapsed time, and every dropped item is listed."""
import importlib.util
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_drop_order_is_fixed(bench):
    d = bench.DROP_AT
    # a lower share of the budget = dropped sooner as time runs out: the calibration mini-sweep, then
    # config #4's tail sizes, then the grid sweep
    assert d["cost_model_fit"] < d["config4_tail"] < d["grid_sweep"] < bench.COMPANION_AT < 1.0


def test_budget_allows_then_drops(bench, monkeypatch):
    agreed = []

    def agree(v):  # every decision goes through the max-over-ranks agreement
        agreed.append(v)
        return v

    b = bench.Budget(100.0, agree)
    monkeypatch.setattr(bench, "_T_START", bench.time.monotonic() - 55.0)  # 55 s spent
    assert b.allow("config5", bench.COMPANION_AT)
    assert not b.allow("cost_model_fit", bench.DROP_AT["cost_model_fit"])
    assert b.allow("config4_tail", bench.DROP_AT["config4_tail"])
    assert [x["item"] for x in b.dropped] == ["cost_model_fit"]
    assert b.dropped[0]["limit_s"] == pytest.approx(100.0 * bench.DROP_AT["cost_model_fit"])
    assert len(agreed) == 3 and all(a >= 55.0 for a in agreed)
    monkeypatch.setattr(bench, "_T_START", bench.time.monotonic() - 99.0)
    for item in ("grid_sweep", "config4_tail", "config3"):
        assert not b.allow(item, bench.DROP_AT.get(item, bench.COMPANION_AT))
    assert [x["item"] for x in b.dropped] == ["cost_model_fit", "grid_sweep", "config4_tail", "config3"]


def test_sizes_of_the_config4_sweep(bench):
    assert bench._x4(4096, 1 << 30) == [4096 << (2 * k) for k in range(10)]
    assert bench.parse_bytes("4K") == 4096 and bench.parse_bytes("1G") == 1 << 30
