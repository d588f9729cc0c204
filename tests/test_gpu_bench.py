"""The driver's bench contract at N > 1, on a 1-GPU box: bench.py under torch.distributed.run with two ranks
sharing device 0 and RCCL in the loop (FLEXAR_BENCH_SHARED_RCCL=1: one NCCL_HOSTID per rank). The tuner's pick
is rejected on purpose (FLEXAR_BENCH_REJECT_FIRST=1), so the final-check fallback chain must hand over to the
runner-up on a rebuilt communicator, which must still pass its connect-time self-test on every IPC family, and
the one JSON line must carry the contract's keys and name the rejection."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _diag(r, name):
    """Why a bench run failed: its whole output is kept under gpurun_out/ (merged back from the GPU box), and
    the message carries the bench's last progress lines and every error-looking line, not just the tail
    (the tail of an aborted rank is RCCL's crash dump)."""
    text = (r.stdout or "") + "\n" + (r.stderr or "")
    try:
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        with open(os.path.join(REPO, "gpurun_out", f"test_bench_{name}.log"), "w") as f:
            f.write(text)
    except OSError:
        pass
    lines = text.splitlines()
    progress = [ln for ln in lines if ln.startswith("[bench]")][-15:]
    errors = [ln for ln in lines if any(k in ln.lower() for k in ("error", "fault", "illegal", "abort", "exception"))]
    return "\n".join(["-- progress:"] + progress + ["-- errors:"] + errors[:25] + ["-- tail:", text[-1500:]])


def _keep(r, name):
    """Every bench run's whole output under gpurun_out/ (the per-rank phase timelines)."""
    try:
        os.makedirs(os.path.join(REPO, "gpurun_out", "bench_tests"), exist_ok=True)
        with open(os.path.join(REPO, "gpurun_out", "bench_tests", f"{name}.log"), "w") as f:
            f.write((r.stdout or "") + "\n" + (r.stderr or ""))
    except OSError:
        pass


def test_bench_json_and_fallback_chain_two_ranks(cuda):
    env = dict(os.environ, FLEXAR_BENCH_SHARED_GPU="1", FLEXAR_BENCH_SHARED_RCCL="1", FLEXAR_BENCH_REJECT_FIRST="1",
               FLEXAR_NO_BUILD="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--size-mb", "16", "--no-calibrate", "--no-small"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=REPO)
    _keep(r, "fallback")
    assert r.returncode == 0, _diag(r, "fallback")
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["value"] == out["busbw_GBps"] > 0
    rejected = out["tuner"]["rejected_after_tuning"]
    assert len(rejected) == 1 and "FLEXAR_BENCH_REJECT_FIRST" in next(iter(rejected.values())), rejected
    assert out["fallback"] is None and out["config"]["algorithm"] not in rejected, out["config"]
    assert out["readiness"]["disabled"] == "", out["readiness"]  # the rebuilt communicator kept every family
    assert out["hbm_TBps_per_rank"] and 0 < out["hbm_TBps_per_rank"] < 10, out["hbm_TBps_per_rank"]


def _bench(extra_env, args, timeout=300):
    env = dict(os.environ, FLEXAR_BENCH_SHARED_GPU="1", FLEXAR_BENCH_SHARED_RCCL="1", FLEXAR_NO_BUILD="1", **extra_env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", *args]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=REPO)
    _keep(r, "sections_" + "_".join(sorted(extra_env)) if extra_env else "sections")
    assert r.returncode == 0, _diag(r, "sections")
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_baseline_config_sections(cuda):
    """Configs #3 / #4 / #5 ride along in the same JSON line (small buffers here; the driver's run uses the
    BASELINE sizes): each next to RCCL, with correctness."""
    out = _bench({}, ["--size-mb", "16", "--config3-mb", "16", "--config4-max", "1M", "--config5-mb", "16",
                      "--no-calibrate"])
    c3, c4, c5 = out["config3"], out["config4"], out["config5"]
    assert set(c3["variants"]) == {"rhd+pull+f32", "rhd+pull+rw", "auto"}, c3
    for v in c3["variants"].values():
        assert v.get("correct") is True and v["busbw_GBps"] > 0, c3
    assert c3["rccl"]["busbw_GBps"] > 0
    sizes = [r["bytes"] for r in c4["rows"]]
    assert sizes == [4096, 16384, 65536, 262144, 1048576], c4
    assert all(r["correct"] is True and r["rccl_busbw"] for r in c4["rows"]), c4
    assert c5["correct"] is True and c5["max_rel_err"] < 0.13 and c5["rccl_fp32_avg_busbw_GBps"] > 0, c5
    assert out["dropped"] is None and out["bench_wall_s"] > 0 and out["budget_s"] == 400
    assert out["readiness"]["calibration"]["source"] in ("measured", "cache"), out["readiness"]
    if out["zero_copy"]["registered"]:  # the automatic choice on registered buffers, as it ran (last_spec)
        assert "+zc" in (out["cost_model"].get("registered_choice") or ""), out["cost_model"]


def test_bench_budget_drops_in_order(cuda):
    """A budget that is already spent: every optional item and companion section is dropped and listed,
    the headline still runs and the JSON line still comes out."""
    out = _bench({"FLEXAR_BENCH_BUDGET_S": "1"}, ["--size-mb", "16", "--config3-mb", "16", "--config4-max", "1M",
                                                   "--config5-mb", "16"])
    items = [d["item"] for d in out["dropped"]]
    assert items[0] == "grid_sweep" and "cost_model_fit" in items, items
    for k in ("config3", "config4", "config5", "small_msg"):
        assert k in items and k not in out, (k, items)
    assert out["value"] > 0 and out["cost_model_fit"] is None and out["bench_wall_s"] > 1


def test_bench_json_names_a_recovered_selftest_family(cuda):
    """rank 1 starts the first self-test family 1.5 s late (FLEXAR_SELFTEST_SKEW), past its
    peer's 300 ms self-test watchdog: the fence family fails once and passes the second pass. The ranks
    share one GPU, so it is kept - and the bench JSON says so (readiness.selftest_recovered, the notes and
    the per-creation record); nothing is silent."""
    out = _bench({"FLEXAR_SELFTEST_SKEW": "1:1500", "FLEXAR_SELFTEST_TIMEOUT_MS": "300"},
                 ["--size-mb", "4", "--no-configs", "--no-calibrate", "--no-small", "--no-tune", "--algo", "flat+pull"])
    rd = out["readiness"]
    assert rd["selftest_recovered"] == ["fence"] and rd["selftest_flaky"] == [], rd
    assert rd["disabled"] == "", rd
    assert rd["selftest_notes"] and any("flat+pull" in v for v in rd["selftest_notes"].values()), rd
    assert rd["creations"][0]["selftest_recovered"] == ["fence"], rd
    assert rd["host_page"]["joined"] is True and rd["host_page"]["verified_shared"] is True, rd
    assert out["value"] > 0


def test_bench_n1_line_carries_the_group_executor_section(cuda):
    """The driver's N = 1 line (no launcher): besides the headline it carries the 8-ranks-in-one-launch executor
    section, every schedule family of the 8-GPU node (the link-balanced channelled trees among them) exact on
    integer data, with a time and an effective HBM rate."""
    env = dict(os.environ, FLEXAR_NO_BUILD="1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--no-reduce-kernel"], env=env, capture_output=True, text=True, timeout=240, cwd=REPO)
    _keep(r, "n1_group_executor")
    assert r.returncode == 0, _diag(r, "n1_group_executor")
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["value"] == 0.0
    rows = {row["spec"]: row for row in out["group_executor"]["rows"]}
    assert {"rhd+pull", "rhd:7+pull", "tree:4,2:7+pull", "flat+pull"} <= set(rows), rows
    for spec, row in rows.items():
        assert row.get("exact") is True and row["us"] > 0 and 0 < row["eff_hbm_TBps"] < 10, (spec, row)
