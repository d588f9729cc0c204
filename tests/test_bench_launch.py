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
