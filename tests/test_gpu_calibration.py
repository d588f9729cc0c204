"""Connect-time calibration and probe agreement on the device.

Separate processes on one GPU (IPC, gloo bootstrap), like tests/test_gpu_ipc.py:
* the first communicator measures calib_points() and installs identical constants on every rank (same
  model hash); a second communicator of the same shape loads them from the on-disk cache; FLEXAR_CALIB=0
  leaves the default model; the calibrated selector's choice still produces exact results;
* a rank whose calibration scratch is unavailable (FLEXAR_TEST_CALIB_FAIL, test-only) still makes every
  collective call of the calibration: every rank reports "failed", keeps the default model, and later calls
  stay in step;
* a rank that reports a different link class for its peers (FLEXAR_TEST_PROBE, test-only) makes EVERY
  rank fail at connect with a message naming the disagreement - not a watchdog timeout later.
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, calib_dir, mode, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16",
                          FLEXAR_TIMEOUT_MS="20000", FLEXAR_CALIB_DIR=calib_dir)
        if mode == "probe":
            os.environ["FLEXAR_TEST_PROBE"] = "1:class=pcie"
        if mode == "scratch":
            os.environ["FLEXAR_TEST_CALIB_FAIL"] = str(world - 1)  # that rank's calibration scratch "fails"
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from allreduce_over_mpi_amd import _native as nv
        from allreduce_over_mpi_amd.parallel import Communicator

        out = {}
        if mode == "probe":
            try:
                Communicator(workspace_bytes=64 << 20)
                out["error"] = None
            except nv.FlexarError as e:
                out["error"] = str(e)
        elif mode == "scratch":
            os.environ["FLEXAR_CALIB"] = "force"
            comm = Communicator(workspace_bytes=64 << 20)
            out["cal"] = comm.calibration
            dev = torch.device("cuda", 0)
            errs = []
            for algo in (None, "ll", "oneshot", "flat", "ring"):  # epochs still in lockstep on every rank
                for n in (1000, 1 << 18):
                    x = (torch.arange(n, device=dev, dtype=torch.int32) % 977 + rank).float()
                    y = comm.all_reduce(x.clone(), algo=algo)
                    want = (torch.arange(n, device=dev, dtype=torch.int32) % 977).float() * world + world * (world - 1) / 2
                    errs.append(float((y - want).abs().max().item()))
            out["err"] = max(errs)
            comm.check()
            comm.close()
        else:
            for i, calib in enumerate(("1", "1", "0")):
                os.environ["FLEXAR_CALIB"] = calib
                try:  # no caller barrier between close() and the next communicator: the library agrees on it
                    comm = Communicator(workspace_bytes=128 << 20)
                except Exception as e:
                    raise RuntimeError(f"creating communicator {i} (FLEXAR_CALIB={calib}) failed") from e
                out[f"cal{i}"] = comm.calibration
                out[f"hash{i}"] = int(comm._lib.flexar_comm_model_hash(comm._h))
                out[f"topo{i}"] = comm.topology()
                out[f"bucket{i}"] = (comm.recommended_bucket_bytes(0.9), comm.recommended_bucket_bytes(0.9, True))
                # the calibrated model's own choice at a few sizes: exact integer sums
                dev = torch.device("cuda", 0)
                errs = []
                for n in (1000, 1 << 18, 1 << 22):
                    x = (torch.arange(n, device=dev, dtype=torch.int32) % 977 + rank).float()
                    y = comm.all_reduce(x.clone())
                    want = (torch.arange(n, device=dev, dtype=torch.int32) % 977).float() * world + world * (world - 1) / 2
                    errs.append(float((y - want).abs().max().item()))
                    out.setdefault(f"choice{i}", []).append(comm.describe(n, torch.float32).split(" ")[0])
                out[f"err{i}"] = max(errs)
                comm.check()
                comm.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out, None))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, None, traceback.format_exc()))


def _run(world, mode, calib_dir):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, calib_dir, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, res, err = q.get(timeout=240)
        assert err is None, f"rank {rank} failed:\n{err}"
        out[rank] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_calibration_measures_caches_and_agrees(cuda, tmp_path, world):
    out = _run(world, "calib", str(tmp_path))
    r0 = out[0]
    assert r0["cal0"]["source"] == "measured", r0["cal0"]
    assert r0["cal1"]["source"] == "cache", r0["cal1"]
    assert r0["cal2"]["source"] == "off"
    for r in range(world):
        assert out[r]["hash0"] == r0["hash0"] and out[r]["hash1"] == r0["hash1"]  # identical model everywhere
        assert out[r]["choice0"] == r0["choice0"]
        assert out[r]["bucket0"] == r0["bucket0"] and out[r]["bucket1"] == r0["bucket1"]  # same bucket everywhere
        for i in range(3):
            assert out[r][f"err{i}"] == 0.0, (r, i, out[r])
            assert out[r][f"topo{i}"]["links_agreed"]
    for b in r0["bucket0"]:
        assert (1 << 20) <= b <= (1 << 30) and b % (1 << 20) == 0, r0["bucket0"]
    assert r0["hash0"] == r0["hash1"] != r0["hash2"]  # the cache reproduces the measured constants exactly
    cal = r0["cal0"]
    assert len(cal["rows"]) >= 6 and all(row[2] > 0 for row in cal["rows"])
    assert cal["median_rel_err"] < 0.5, cal
    assert os.path.exists(cal["path"])


def test_probe_disagreement_fails_at_connect(cuda, tmp_path):
    out = _run(2, "probe", str(tmp_path))
    for r in range(2):
        e = out[r]["error"]
        assert e and "disagree on the machine shape" in e, (r, e)


@pytest.mark.parametrize("world", [2, 4])
def test_calibration_local_failure_keeps_ranks_in_step(cuda, tmp_path, world):
    out = _run(world, "scratch", str(tmp_path))
    for r in range(world):
        assert out[r]["cal"]["source"] == "failed", (r, out[r]["cal"])
        assert out[r]["err"] == 0.0, (r, out[r])
