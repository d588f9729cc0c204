"""Gradient-bucket size from the calibrated selector (utils/perf.py recommend_bucket_bytes,
Communicator.recommended_bucket_bytes): the smallest bucket whose allreduce reaches a fraction of the
asymptotic bandwidth on this node's links. The reference has no training integration;
DDP's 25 MiB default was tuned for other interconnects."""
import pytest

from allreduce_over_mpi_amd import _native as nv
from allreduce_over_mpi_amd.utils.perf import recommend_bucket_bytes

MiB = 1 << 20


def test_alpha_beta_knee():
    alpha, bw = 20.0, 400e3  # us, bytes per us (400 GB/s)
    cost = lambda b: alpha + b / bw  # noqa: E731
    got = recommend_bucket_bytes(cost, 0.9)
    hi = float(1 << 30)
    target = 0.9 * hi / cost(hi)
    assert got % MiB == 0
    assert got / cost(got) >= target
    assert (got - MiB) / cost(got - MiB) < target
    # closed form: b / (alpha + b / bw) = target  <=>  b = target * alpha / (1 - target / bw)
    assert abs(got - target * alpha / (1 - target / bw)) <= MiB


def test_bounds_and_monotone_in_efficiency():
    cost = lambda b: 15.0 + b / 300e3  # noqa: E731
    sizes = [recommend_bucket_bytes(cost, e) for e in (0.5, 0.8, 0.9, 0.95, 0.99)]
    assert sizes == sorted(sizes) and sizes[0] >= MiB and sizes[-1] <= 1 << 30
    assert recommend_bucket_bytes(lambda b: 1.0 + b, 0.9) == MiB  # bandwidth-bound everywhere: the floor
    with pytest.raises(ValueError):
        recommend_bucket_bytes(cost, 1.5)


def test_with_the_native_model_at_eight_ranks():
    """The default xGMI model at N = 8 (7 links): the 90 % knee lies between 1 MiB and 1 GiB."""
    def auto_cost(b):
        return nv.model_cost_us(nv.select_plan(8, b, links=7), 8, b)

    got = recommend_bucket_bytes(auto_cost, 0.9)
    assert MiB <= got <= 1 << 30
    assert got / auto_cost(got) >= 0.9 * (1 << 30) / auto_cost(float(1 << 30))
