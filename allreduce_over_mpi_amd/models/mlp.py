"""Data-parallel demo model: the training workload the reference's allreduce
exists to serve (DP gradient allreduce is the implicit use case
of MPI_Allreduce_FT's interposer mode, mpi_mod.hpp:1170).

``MLP`` is a small fully connected network; ``dp_smoke_step`` runs one data
parallel step with two replicas on one GPU whose flattened gradient buckets are
averaged by the flexar executor kernel (LocalGroup, in one launch), and checks
the result against the single-replica full-batch gradient.
"""
from __future__ import annotations

import torch
import torch.nn as nn


class MLP(nn.Module):
    def __init__(self, d_in=64, d_hidden=256, d_out=16, layers=3):
        super().__init__()
        dims = [d_in] + [d_hidden] * (layers - 1) + [d_out]
        mods = []
        for i in range(len(dims) - 1):
            mods.append(nn.Linear(dims[i], dims[i + 1]))
            if i < len(dims) - 2:
                mods.append(nn.GELU())
        self.net = nn.Sequential(*mods)

    def forward(self, x):
        return self.net(x)


def flat_grads(model: nn.Module) -> torch.Tensor:
    return torch.cat([p.grad.reshape(-1) for p in model.parameters()])


def dp_smoke_step(device, nranks: int = 2, batch: int = 32, seed: int = 0) -> dict:
    from ..parallel.comm import LocalGroup

    torch.manual_seed(seed)
    ref = MLP().to(device)
    replicas = [MLP().to(device) for _ in range(nranks)]
    for r in replicas:
        r.load_state_dict(ref.state_dict())
    x = torch.randn(batch * nranks, 64, device=device)
    y = torch.randn(batch * nranks, 16, device=device)
    loss_fn = nn.MSELoss()

    # reference: one replica, full batch
    loss_fn(ref(x), y).backward()
    g_ref = flat_grads(ref)

    # data parallel: each replica its shard, gradients averaged by flexar
    buckets = []
    for i, m in enumerate(replicas):
        sl = slice(i * batch, (i + 1) * batch)
        loss = loss_fn(m(x[sl]), y[sl])
        loss.backward()
        buckets.append(flat_grads(m).contiguous())
    grp = LocalGroup(nranks, workspace_bytes=8 << 20)
    try:
        outs = grp.all_reduce(buckets, op="avg", algo="flat")
        torch.cuda.synchronize()
        grp.check()
    finally:
        grp.close()
    err = max((o - g_ref).abs().max().item() for o in outs)
    scale = g_ref.abs().max().item()
    assert err <= 1e-5 * max(1.0, scale), f"DP gradient mismatch: {err}"
    # optimizer step on every replica with the averaged gradient
    for m, g in zip(replicas, outs):
        off = 0
        with torch.no_grad():
            for p in m.parameters():
                n = p.numel()
                p -= 0.01 * g[off:off + n].view_as(p)
                off += n
    return {"params": int(g_ref.numel()), "max_grad_err": err, "ranks": nranks}
