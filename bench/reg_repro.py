#!/usr/bin/env python3
"""Registration of several large buffers by N processes sharing one GPU (diagnostic for registration
hangs): each rank allocates REGR_COUNT tensors of REGR_MIB MiB (torch allocator, or hipMalloc'd with
REGR_RAW=1) and registers them one after the other, printing progress with timestamps."""
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), FLEXAR_MAX_GRID="16")
    import faulthandler

    faulthandler.dump_traceback_later(60, repeat=True)
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from allreduce_over_mpi_amd.parallel import Communicator

    comm = Communicator(workspace_bytes=64 << 20)
    mib = int(os.environ.get("REGR_MIB", "1024"))
    n = int(os.environ.get("REGR_COUNT", "3"))
    dt = torch.bfloat16 if os.environ.get("REGR_BF16", "1") == "1" else torch.float32
    count = (mib << 20) // torch.tensor([], dtype=dt).element_size()
    ts = []
    mode = os.environ.get("REGR_MODE", "carved")
    if mode == "raw":  # a hipMalloc'd allocation of 2 x REGR_MIB through flexar, registered by pointer
        import ctypes

        lib = comm._lib
        lib.flexar_device_alloc.restype = ctypes.c_void_p
        lib.flexar_device_alloc.argtypes = [ctypes.c_size_t]
        nbytes = 2 * (mib << 20)
        ptr = lib.flexar_device_alloc(nbytes)
        if os.environ.get("REGR_TOUCH", "0") == "1":  # populate the allocation before exporting it
            hip = ctypes.CDLL("libamdhip64.so")
            hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
            hip.hipDeviceSynchronize()
            assert hip.hipMemset(ptr, 0, nbytes) == 0
            hip.hipDeviceSynchronize()
        blob = ctypes.create_string_buffer(int(lib.flexar_reg_handle_size()))
        assert lib.flexar_reg_export(comm._h, ptr, nbytes, blob) == 0
        rows = comm._exchange(bytes(blob.raw))
        rid = ctypes.c_int(0)
        t0 = time.time()
        rc = lib.flexar_reg_open(comm._h, ptr, nbytes, b"".join(rows), ctypes.byref(rid))
        print(f"[r{rank}] raw {nbytes} B registration rc={rc} in {time.time() - t0:.2f} s", flush=True)
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        return
    if mode == "view":  # two halves of one allocation
        big = torch.empty(2 * count, device="cuda", dtype=dt)
        ts = [big[:count], big[count:]]
    elif mode == "whole2g":  # one allocation of twice the size, registered whole
        ts = [torch.empty(2 * count, device="cuda", dtype=dt)]
    else:
        for i in range(n):
            if mode == "carved" and i == 1:
                tmp = ts[0].float()  # a freed larger block the allocator may carve the next tensors from
                del tmp
            ts.append(torch.empty(count, device="cuda", dtype=dt))
    for i, t in enumerate(ts):
        t0 = time.time()
        comm.register(t)
        print(f"[r{rank}] registered {i} ({mib} MiB) in {time.time() - t0:.2f} s", flush=True)
    x = ts[0][:1 << 20]
    x.fill_(1)
    comm.all_reduce(x, algo="flat+zc+push")
    torch.cuda.synchronize()
    print(f"[r{rank}] allreduce ok: {float(x[0])}", flush=True)
    comm.close()
    dist.barrier()
    dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp

    world = int(os.environ.get("REGR_RANKS", "4"))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=worker, args=(r, world, port)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join()
    sys.exit(max(abs(p.exitcode or 0) for p in ps))


if __name__ == "__main__":
    main()
