"""Message transport on the GPU box: RCCL is resolved at run time (dlopen of the process's librccl) and the
device side of a message plan (local executor segments, arena, grouped ncclSend/ncclRecv) runs. A 1-GPU
box allows one RCCL rank per GPU and host, so the multi-rank transport runs in
tests/test_gpu_msg_shared.py (ranks on one GPU posing as separate hosts through NCCL_HOSTID) and
tests/test_gpu_multidevice.py (2+ GPUs); the message plans themselves are validated on the CPU
(tests/test_msg_plan.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_rccl_resolved_at_run_time(cuda):
    from allreduce_over_mpi_amd import _native as nv

    assert nv.lib().flexar_rccl_available() == 1
    import ctypes

    uid = ctypes.create_string_buffer(128)
    nv.check(nv.lib().flexar_rccl_unique_id(uid, 128), "unique_id")
    assert any(uid.raw)


def test_msg_transport_single_rank(cuda):
    """One-rank RCCL communicator: the '+rccl' route through run_msg (plan build, arena, executor segment)."""
    from allreduce_over_mpi_amd.parallel import Communicator

    c = Communicator(rank=0, world_size=1, workspace_bytes=16 << 20)
    c._init_msg(lambda b: [b])
    assert c.topology()["rccl"] is True
    for n in (1, 4099, 1 << 20):
        x = torch.randn(n, device=cuda)
        y = c.all_reduce(x, out=torch.empty_like(x), algo="flat+rccl")
        z = c.all_reduce(x.clone(), op="avg", algo="ring+rccl")
        torch.cuda.synchronize()
        assert torch.equal(y, x) and torch.equal(z, x)
    c.check()
    c.close()
