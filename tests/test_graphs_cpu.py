"""CapturedAllReduce argument handling on the host (the capture itself runs in tests/test_gpu_ipc.py)."""
import pytest


class _FakeComm:
    device = 0

    def describe(self, count, dtype):
        return "dma grid=1 pieces=1" if count >= 1 << 20 else "ll grid=1 pieces=1"


def test_mismatched_lists_rejected_before_any_device_work():
    import torch

    from allreduce_over_mpi_amd.parallel import CapturedAllReduce

    ts = [torch.empty(4), torch.empty(8)]
    with pytest.raises(ValueError):
        CapturedAllReduce(_FakeComm(), ts, outs=[None])
    with pytest.raises(ValueError):
        CapturedAllReduce(_FakeComm(), ts, algo=["ll"])


def test_dma_is_never_captured():
    """The copy-engine path bakes the host's epoch into its copies: requested or selected, it is replaced by
    the executor's flat exchange before warm-up, so the replayed graph never contains it."""
    import torch

    from allreduce_over_mpi_amd.parallel.graphs import CapturedAllReduce

    cap = CapturedAllReduce.__new__(CapturedAllReduce)
    cap.comm = _FakeComm()
    small, big = torch.empty(16), torch.empty(1 << 20)
    assert cap._capturable(small, "dma") == "flat+pull"
    assert cap._capturable(small, "dma+wt") == "flat+pull"
    assert cap._capturable(big, None) == "flat+pull"      # the selector would pick dma
    assert cap._capturable(small, None) is None           # the selector's choice (ll) is capturable
    assert cap._capturable(small, "ring:2") == "ring:2"
