"""The crash report's device progress words on a real GPU: executor workgroup 0 stores the epoch it starts and
finishes for launches of at least FLEXAR_PROGRESS_MIN_BYTES (1 MiB); small calls skip the two system-scope stores
(0.4-0.7 us of a small call, profiles/r6_latency) but still leave their breadcrumb. A child makes two 4 MiB calls
and one 8 KiB call, then dumps the report."""
import os
import re
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import sys
    sys.path.insert(0, {repo!r})
    import torch
    from allreduce_over_mpi_amd import _native as nv
    from allreduce_over_mpi_amd.parallel import Communicator
    comm = Communicator(rank=0, world_size=1)
    x = torch.ones(1 << 20, device="cuda")
    for _ in range(2):
        comm.all_reduce(x)
    comm.all_reduce(torch.ones(2048, device="cuda"))
    torch.cuda.synchronize()
    nv.lib().flexar_crash_report_dump(b"progress test")
""")


def test_progress_words_for_large_launches_only(cuda):
    env = dict(os.environ, FLEXAR_NO_BUILD="1")
    env.pop("FLEXAR_CRASH_REPORT", None)
    env.pop("FLEXAR_PROGRESS", None)
    r = subprocess.run([sys.executable, "-c", CHILD.format(repo=REPO)], env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    m = re.search(r"started epoch (\d+), finished epoch (\d+)", r.stderr)
    assert m, r.stderr[-3000:]
    started, finished = int(m.group(1)), int(m.group(2))
    assert started == finished >= 2, (started, finished)
    launches = [ln for ln in r.stderr.splitlines() if " launch " in ln and "epoch" in ln]
    assert len(launches) >= 3, r.stderr[-3000:]  # the small call is in the breadcrumbs all the same
