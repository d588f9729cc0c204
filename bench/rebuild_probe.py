#!/usr/bin/env python3
"""Communicator rebuilt in the same processes (what bench.py's tuner and final-check fallback do after a
failure): N processes on one GPU create, use and close a Communicator several times in a row; each round
reports the connect-time self-test verdict and an exact flat allreduce, with and without registered
buffers. A rebuilt communicator must pass exactly like the first one.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 bench/rebuild_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist

    os.environ.setdefault("FLEXAR_MAX_GRID", "16")
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    transport = os.environ.get("RBP_TRANSPORT", "ipc")
    if transport == "rccl":  # RCCL with several ranks on one GPU: one NCCL_HOSTID per rank (loopback sockets)
        os.environ.update(NCCL_HOSTID=f"rbp-rank{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    from allreduce_over_mpi_amd.parallel.comm import Communicator

    ws = int(os.environ.get("RBP_WS_MIB", "1088")) << 20
    n = 1 << 22
    x = torch.empty(n, device="cuda")
    y = torch.empty_like(x)
    rows = []
    for rnd in range(int(os.environ.get("RBP_ROUNDS", "3"))):
        comm = Communicator(workspace_bytes=ws, transport=transport)
        reg = os.environ.get("RBP_REGISTER", "1") == "1"
        if reg:
            comm.register_many([x, y])
        x.fill_(float(rank + 1))
        ok = True
        specs = os.environ.get("RBP_SPECS", "flat+pull,flat+zc+push,dma").split(",")
        for spec in specs + (["flat+rccl"] if transport == "rccl" else []):
            if "+zc" in spec and not reg:
                continue
            y.zero_()
            comm.all_reduce(x, out=y, algo=spec)
            torch.cuda.synchronize()
            ok = ok and bool((y == world * (world + 1) / 2).all().item())
        topo = comm.topology()
        rows.append({"round": rnd, "rank": rank, "disabled": topo["disabled"], "flat_ok": ok, "registered": reg,
                     "zc_ok": getattr(comm, "_zc_ok", None)})
        comm.close()
        torch.cuda.synchronize()
        dist.barrier()
    for r in rows:
        print(json.dumps(r), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
