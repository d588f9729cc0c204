"""The CPython fast-call entry (csrc/python/fastcall.c) on the host: it is built with the library, forwards
every argument to the C API unchanged (a null communicator is rejected by the library itself), and rejects
malformed calls with Python exceptions instead of crashing."""
import pytest


@pytest.fixture(scope="module")
def nv():
    from allreduce_over_mpi_amd import _native as nv

    nv.lib()
    return nv


def test_fastcall_module_loaded(nv):
    assert nv.FAST is not None, "fast-call module missing: run __graft_entry__.build()"
    assert nv.AR and nv.RS and nv.AG


def test_fastcall_forwards_to_the_c_api(nv):
    # null communicator: the library's own argument check answers, through the fast path
    assert nv.FAST.ar(nv.AR, 0, 0, 0, 16, 0, 0, 0, b"ring", 1.0) == 1
    assert "null communicator" in nv.last_error()
    assert nv.FAST.rs(nv.RS, 0, 0, 0, 16, 0, 0, 0, None) != 0
    assert nv.FAST.ag(nv.AG, 0, 0, 0, 16, 0, 0, None) != 0


def test_fastcall_rejects_malformed_calls(nv):
    with pytest.raises(TypeError):
        nv.FAST.ar(nv.AR, 0, 0)
    with pytest.raises(TypeError):
        nv.FAST.ar(nv.AR, 0, 0, 0, 16, 0, 0, 0, "not-bytes", 1.0)
    with pytest.raises(TypeError):
        nv.FAST.ar(nv.AR, 0, 0, 0, 16, 0, 0, 0, None, "not-a-float")
    with pytest.raises(ValueError):
        nv.FAST.ar(0, 0, 0, 0, 16, 0, 0, 0, None, 1.0)  # null entry point


def test_enum_memos_match_the_slow_path(nv):
    import torch

    from allreduce_over_mpi_amd.parallel import comm as cm

    for dt in (torch.float32, torch.bfloat16, torch.float16, torch.int32, torch.uint8, torch.bool):
        assert cm._dt(dt) == nv.dtype_code(dt)
        assert cm._dt(dt) == nv.dtype_code(dt)  # memoised
    for op in ("sum", "avg", "max", "band"):
        assert cm._op(op) == nv.op_code(op)
    assert cm._algo(None) is None and cm._algo("ring") == b"ring" and cm._algo("") is None
