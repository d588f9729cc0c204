"""Message transport plans (csrc/include/flexar/msg_plan.hpp): the IPC schedules rewritten as local
executor segments + grouped send/recv - what the RCCL transport ("+rccl", and every call when IPC mapping
is unavailable) posts, and what the MPI point-to-point engine coalesces (shared msg_regions).

Run on the CPU through per-pair in-order mailboxes (NCCL matches a rank pair's sends/receives in order):
every schedule of the planner gives the exact sum; messages are one per (peer, stage) and every rank
moves the bandwidth-optimal 2 (N - 1) / N of the buffer (the reference's verified per-call message
statistics, SURVEY.md section 2.3, coalesced per peer and stage)."""
import numpy as np
import pytest

from allreduce_over_mpi_amd import _native as nv

CASES = [(2, "flat"), (3, "flat"), (4, "ring"), (5, "ring"), (8, "ring:2"), (8, "rhd"), (8, "tree:2,4"),
         (8, "tree:4,2"), (8, "flat"), (6, "tree:3,2"), (7, "tree:2,3"), (4, "oneshot"), (8, "ll"), (4, "dma"),
         (16, "flat"), (12, "tree:3,4")]


@pytest.mark.parametrize("n,spec", CASES)
@pytest.mark.parametrize("count", [1, 35, 10007])
def test_msg_plan_exact_sum(n, spec, count):
    ins = [np.random.default_rng(100 * r + count).integers(-99, 99, count).astype(np.int32) for r in range(n)]
    outs = nv.simulate_msg(spec, ins, ncalls=2)
    want = np.sum(ins, axis=0)
    for o in outs:
        np.testing.assert_array_equal(o, want)


@pytest.mark.parametrize("op,dtype", [("avg", "float32"), ("max", "float32"), ("band", "int64"), ("prod", "float64")])
def test_msg_plan_ops(op, dtype):
    n = 4
    rng = np.random.default_rng(7)
    ins = [(rng.integers(1, 4, 4099) if dtype == "int64" else rng.random(4099) + 0.5).astype(dtype) for _ in range(n)]
    outs = nv.simulate_msg("tree:2,2", ins, op=op)
    stack = np.stack(ins)
    want = {"avg": lambda: stack.mean(0), "max": lambda: stack.max(0),
            "band": lambda: np.bitwise_and.reduce(stack, 0), "prod": lambda: stack.prod(0)}[op]()
    for o in outs:
        np.testing.assert_allclose(o, want, rtol=1e-6)


@pytest.mark.parametrize("n,spec,msgs", [(8, "flat", 14), (8, "ring", 14), (8, "rhd", 6), (8, "tree:2,4", 8),
                                         (8, "tree:4,2", 8), (4, "flat", 6), (2, "flat", 2)])
def test_messages_are_coalesced_and_bandwidth_optimal(n, spec, msgs):
    count = 1 << 20  # divisible: no tail blocks
    for r in range(n):
        m = nv.msg_plan(spec, r, n, count, "float32")
        assert m["messages"] == msgs, m  # one per (peer, stage): the reference posts one Isend per block
        assert m["message_bytes"] == 2 * (n - 1) * count * 4 // n  # 2 (N-1)/N of the buffer, every schedule
        groups = [s for s in m["steps"] if "send" in s]
        # every group posts sends AND receives together (no rank order can deadlock)
        assert all(g["send"] and g["recv"] for g in groups), m["steps"]


def test_zero_copy_sends_and_receives():
    m = nv.msg_plan("flat", 0, 4, 1 << 20, "float32")
    first, second = [s for s in m["steps"] if "send" in s]
    assert all(src == "in" for _, _, src in first["send"])   # reduce-scatter blocks leave straight from IN
    assert all(src == "out" for _, _, src in second["send"])  # the reduced block leaves straight from OUT
    assert m["zero_copy"] == 6


@pytest.mark.parametrize("n,spec,min_zc", [(8, "rhd", 2), (8, "tree:2,4", 2), (8, "tree:4,2", 2), (6, "tree:2,3", 2),
                                           (6, "tree:3,2", 2)])
def test_tree_stage_payloads_are_contiguous(n, spec, min_zc):
    """Digit-reversed block placement (planner.hpp build_tree): each (stage, peer) payload is one span, so
    the stage-0 reduce-scatter leaves straight from IN and every receive lands in place (no inbox copies:
    each executor segment holds only the schedule's own ops)."""
    count = 3 << 16
    for r in range(n):
        m = nv.msg_plan(spec, r, n, count, "float32")
        groups = [s for s in m["steps"] if "send" in s]
        assert all(src == "in" for _, _, src in groups[0]["send"]), groups[0]
        assert m["zero_copy"] >= min_zc, m
    # and the schedules still compute the exact sum through the message transport (uneven tail blocks)
    ins = [np.arange(5003, dtype=np.int32) * (r + 1) for r in range(n)]
    want = np.arange(5003, dtype=np.int32) * (n * (n + 1) // 2)
    for o in nv.simulate_msg(spec, ins):
        assert (o == want).all()


def test_pull_schedules_are_rewritten_to_push():
    # a pull all-gather reads peer memory; the message plan runs the push form of the same tree
    ins = [np.full(999, r + 1, np.int32) for r in range(4)]
    for o in nv.simulate_msg("tree:2,2+pull", ins):
        assert (o == 10).all()
