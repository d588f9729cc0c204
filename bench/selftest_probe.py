"""Debug driver: N processes on one GPU build a Communicator (probe + self-test) and report timings."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist

    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    from allreduce_over_mpi_amd.parallel import Communicator

    t0 = time.time()
    print(f"[r{rank}] creating", flush=True)
    comm = Communicator(workspace_bytes=32 << 20)
    print(f"[r{rank}] ready in {time.time() - t0:.2f}s failed={comm.selftest_failed} {comm.topology()}", flush=True)
    x = torch.full((4096,), float(rank + 1), device="cuda")
    comm.all_reduce(x)
    torch.cuda.synchronize()
    print(f"[r{rank}] allreduce ok: {x[0].item()}", flush=True)
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
