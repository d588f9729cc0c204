"""bench.py's own launcher and per-rank environment, on the CPU.

* `python bench.py --gpus N` with no launcher (WORLD_SIZE unset) starts the N ranks itself - like the
  reference's driver, started by mpiexec and reading MPI_Comm_size (allreduce_over_mpi/benchmark.cpp:48-52)
  - passes rank 0's JSON line through, and exits non-zero if any rank fails;
* one GPU per rank gets no shared-GPU-only setting (hardware-queue cap, grid clamp, per-rank NCCL host id);
  the one-GPU rehearsal gets exactly those.
"""
import json
import os
import sys
import textwrap

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_per_gpu_env_has_no_shared_gpu_settings():
    for world in (1, 2, 4, 8):
        env = {}
        local, shared, shared_rccl = bench.configure_env(world, world - 1, world - 1, env)
        assert (local, shared, shared_rccl) == (world - 1, False, False)
        assert env == {}, env  # no GPU_MAX_HW_QUEUES, no FLEXAR_MAX_GRID, no NCCL_HOSTID


@pytest.mark.parametrize("world,queues,grid", [(2, None, "64"), (4, None, "32"), (8, "2", "16")])
def test_shared_gpu_rehearsal_env(world, queues, grid):
    env = {"FLEXAR_BENCH_SHARED_GPU": "1"}
    local, shared, shared_rccl = bench.configure_env(world, 1, 1, env)
    assert (local, shared, shared_rccl) == (0, True, False)
    assert env.get("GPU_MAX_HW_QUEUES") == queues
    assert env["FLEXAR_MAX_GRID"] == grid
    assert "NCCL_HOSTID" not in env
    env = {"FLEXAR_BENCH_SHARED_GPU": "1", "FLEXAR_BENCH_SHARED_RCCL": "1", "GPU_MAX_HW_QUEUES": "4"}
    bench.configure_env(world, 1, 1, env)
    assert env["NCCL_HOSTID"] == "flexar-bench-rank1" and env["NCCL_SOCKET_IFNAME"] == "lo"
    # a cap, not a default: the GPU box exports HIP's default of 4 explicitly; 1 stays 1
    assert env["GPU_MAX_HW_QUEUES"] == ("2" if world > 4 else "4")
    env = {"FLEXAR_BENCH_SHARED_GPU": "1", "GPU_MAX_HW_QUEUES": "1"}
    bench.configure_env(world, 1, 1, env)
    assert env["GPU_MAX_HW_QUEUES"] == "1"


def _stub(tmp_path, body):
    p = tmp_path / "child.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def test_self_launch_starts_n_ranks_and_passes_rank0_line(tmp_path, capsys):
    child = _stub(tmp_path, """
        import json, os, sys
        r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        assert os.environ["LOCAL_RANK"] == str(r) and os.environ["MASTER_ADDR"] == "127.0.0.1"
        assert int(os.environ["MASTER_PORT"]) > 0
        print("[rank log]", r, file=sys.stderr)
        print("a non-JSON stdout line from rank", r)
        print(json.dumps({"metric": "m", "n_gpus": n, "rank": r, "argv": sys.argv[1:]}))
    """)
    rc = bench.self_launch(4, [child, "--gpus", "4"])
    out = capsys.readouterr().out.strip().splitlines()
    assert rc == 0
    assert len(out) == 1, out  # exactly rank 0's JSON line on stdout
    line = json.loads(out[0])
    assert line == {"metric": "m", "n_gpus": 4, "rank": 0, "argv": ["--gpus", "4"]}


def test_self_launch_fails_when_a_rank_fails(tmp_path, capsys):
    child = _stub(tmp_path, """
        import json, os, sys, time
        r = int(os.environ["RANK"])
        if r == 1:
            sys.exit(3)
        time.sleep(30 if r == 0 else 0)  # rank 0 would wait for its peer: it is stopped instead
        print(json.dumps({"rank": r}))
    """)
    import time

    t0 = time.monotonic()
    rc = bench.self_launch(2, [child])
    assert rc == 3
    assert time.monotonic() - t0 < 20
    assert capsys.readouterr().out.strip() == ""


def test_main_dispatches_to_self_launch_without_touching_the_gpu(monkeypatch):
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "self_launch", lambda n, argv: calls.append((n, argv)) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    assert calls and calls[0][0] == 8 and calls[0][1][1:] == ["--gpus", "8", "--steps", "3"]
    assert calls[0][1][0].endswith("bench.py")
    import torch

    assert not torch.cuda.is_initialized()


class _StubComm:
    """What bench.readiness_record reads from a Communicator."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def topology(self):
        return {"links": 7, "links_local": 7, "selftested": "fence,wt,ll,dma", "disabled": "wt",
                "host_page": True, "host_page_shared": True,
                "peers": [{"rank": 0, "link": "self"}, {"rank": 1, "link": "xgmi"}, {"rank": 2, "link": "xgmi"}]}


def test_readiness_record_reports_what_readiness_did():
    """the bench JSON names recovered / flaky families, every rank's notes (truncated),
    the creation retry, the transport note and the host page, for the final and every earlier communicator."""
    long_note = "x" * 500
    comm = _StubComm(selftest_recovered=[], selftest_flaky=["wt"], selftest_notes={1: ["flat+pull+wt call 0: timeout"],
                                                                                   2: [long_note]},
                     retried="comm_connect: mapping failed", transport_note=None, host_page_note=None,
                     calibration={"source": "measured"}, selftest_failed=["wt"])
    creations = [bench.creation_record(comm, "rccl")]
    rec = json.loads(json.dumps(bench.readiness_record(comm, creations)))  # JSON-serialisable
    for k in ("links", "selftested", "disabled", "peer_links", "selftest_recovered", "selftest_flaky", "selftest_notes",
              "retried", "transport_note", "host_page", "calibration", "creations"):
        assert k in rec, k
    assert rec["selftest_flaky"] == ["wt"] and rec["disabled"] == "wt" and rec["peer_links"] == ["xgmi"]
    assert rec["selftest_notes"]["1"].startswith("flat+pull+wt") and len(rec["selftest_notes"]["2"]) == 300
    assert rec["retried"] == "comm_connect: mapping failed"
    assert rec["host_page"] == {"joined": True, "verified_shared": True, "note": None}
    assert rec["creations"] == [{"transport": "rccl", "retried": "comm_connect: mapping failed",
                                 "selftest_failed": ["wt"], "selftest_recovered": [], "selftest_flaky": ["wt"]}]


def test_selftest_retry_policy_per_gpu_vs_shared():
    """a family that fails once and passes the second pass is kept only when ranks share a
    GPU (a descheduled rank is expected there); with one GPU per rank - the driver's N-GPU bench - it stays
    disabled (flaky). A family that fails twice is disabled either way."""
    from allreduce_over_mpi_amd.parallel.comm import selftest_policy

    fence, wt = 1, 2
    # shared GPU: fence recovered (kept), wt failed twice (disabled)
    assert selftest_policy(fence | wt, wt, shared_gpu=True, mode="") == (wt, fence, 0)
    # one GPU per rank: fence is flaky -> disabled as well
    assert selftest_policy(fence | wt, wt, shared_gpu=False, mode="") == (fence | wt, 0, fence)
    # overrides
    assert selftest_policy(fence, 0, shared_gpu=False, mode="keep") == (0, fence, 0)
    assert selftest_policy(fence, 0, shared_gpu=True, mode="disable") == (fence, 0, fence)
    # nothing failed: nothing disabled
    assert selftest_policy(0, 0, shared_gpu=False, mode="") == (0, 0, 0)
    # the link-class names the probe reports (csrc/include/flexar/readiness.hpp link_name)
    from allreduce_over_mpi_amd.parallel.comm import shares_gpu

    topo = {"peers": [{"rank": 0, "link": "self"}, {"rank": 1, "link": "same-device"}]}
    assert shares_gpu(topo, 0) and not shares_gpu({"peers": [{"rank": 0, "link": "self"},
                                                            {"rank": 1, "link": "xgmi"}]}, 0)
    # the driver's one-GPU-per-rank environment sets no override
    env = {}
    bench.configure_env(8, 3, 3, env)
    assert "FLEXAR_SELFTEST_RETRY" not in env


def test_rehearsal_does_not_report_a_same_node_ratio():
    """with RCCL over loopback sockets (the shared-GPU rehearsal) vs_rccl is null and the RCCL
    figure is labelled loopback; on one GPU per rank both fields are the same-node bar."""
    f = bench.rccl_fields(450.0, 2.25, shared_rccl=True)
    assert f == {"rccl_busbw_GBps": None, "rccl_busbw_GBps_loopback": 2.25, "vs_rccl": None}
    f = bench.rccl_fields(300.0, 250.0, shared_rccl=False)
    assert f == {"rccl_busbw_GBps": 250.0, "vs_rccl": 1.2}
    assert bench.rccl_fields(300.0, None, shared_rccl=False)["vs_rccl"] is None
