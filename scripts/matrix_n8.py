#!/usr/bin/env python3
"""One-off driver (scripts/gpu_r6x.sh): the multi-device acceptance matrix at world 8 with every rank on device 0,
with a heartbeat line every 60 s (the spawned ranks print nothing while they run)."""
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
# the spawned ranks import the package and the test module too
os.environ["PYTHONPATH"] = os.pathsep.join([REPO, os.path.join(REPO, "tests"), os.environ.get("PYTHONPATH", "")])


def main():
    import test_gpu_multidevice as m

    t = time.time()
    stop = threading.Event()

    def beat():
        while not stop.wait(60):
            print(f"... {time.time() - t:.0f} s", flush=True)

    threading.Thread(target=beat, daemon=True).start()
    res = m._run(8, True)
    stop.set()
    print("ran", round(time.time() - t, 1), "s", flush=True)
    wires = {k: v for k, v in res[0].items() if isinstance(k, tuple) and k[0] in ("mx_mismatch", "fp8_emulation_mismatch")}
    print("rank 0 wire checks:", wires, flush=True)
    m._check(res, 8, True)
    print("matrix n8 shared: ok", flush=True)


if __name__ == "__main__":
    main()
