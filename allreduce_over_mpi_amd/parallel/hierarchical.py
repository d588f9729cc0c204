"""Multi-node allreduce: flexar inside each node (xGMI), a cross-node group between nodes.

The reference runs one flat FlexTree over every MPI rank of a 16-host, 340-slot cluster
(allreduce_over_mpi/mpi_config_file, mpi_mod.hpp:952-1111); its inter-host stages move whole blocks
over the NIC. On MI355X nodes the xGMI mesh inside a node is an order of magnitude faster than the
network, so the node boundary becomes the first tree level:

1. intra-node reduce-scatter over xGMI (flexar): local rank l owns shard l (1/L of the buffer);
2. inter-node allreduce of that shard among the ranks with the same local index, one per node
   (RCCL over the NIC by default): each rank ships only S/L bytes across nodes;
3. intra-node all-gather over xGMI (flexar).

This is the torch.distributed counterpart of the MPI layer's hierarchical device allreduce
(csrc/include/flexar/mpi_mod.hpp ``hierarchical_device_allreduce``). Node membership comes from the
ranks' hostnames (contiguous, equal-sized blocks of ranks), or from ``FLEXAR_NODE_SIZE`` / ``node_size``
(virtual nodes, used to test the scheme on one node).
"""
from __future__ import annotations

import os
import socket
from typing import Optional

from .. import _native as nv
from .comm import Communicator


def _node_size(group, world: int) -> int:
    import torch.distributed as dist

    env = int(os.environ.get("FLEXAR_NODE_SIZE", "0") or 0)
    if env > 0:
        return env
    hosts = [None] * world
    dist.all_gather_object(hosts, socket.gethostname(), group=group)
    L = hosts.count(hosts[0])
    if world % L or any(hosts[i] != hosts[(i // L) * L] for i in range(world)) or len(set(hosts)) != world // L:
        raise nv.FlexarError(1, "hierarchical allreduce needs contiguous, equal-sized blocks of ranks per host")
    return L


class HierarchicalCommunicator:
    """Allreduce over ``group`` (default: WORLD) as intra-node flexar RS -> cross-node allreduce -> AG."""

    def __init__(self, group=None, node_size: Optional[int] = None, workspace_bytes: int = 0,
                 cross_backend: Optional[str] = None):
        import torch
        import torch.distributed as dist

        self.group = group
        ranks = dist.get_process_group_ranks(group or dist.group.WORLD)
        self.world = self.world_size = len(ranks)
        self.rank = dist.get_rank(group)
        L = node_size or _node_size(group, self.world)
        if L < 1 or self.world % L:
            raise nv.FlexarError(1, f"node size {L} does not divide the world size {self.world}")
        self.L, self.nodes = L, self.world // L
        self.local_rank, self.node = self.rank % L, self.rank // L
        # every rank creates every subgroup, in the same order (torch.distributed requirement)
        self.local_group = self.cross_group = None
        for n in range(self.nodes):
            g = dist.new_group(ranks[n * L:(n + 1) * L])
            if n == self.node:
                self.local_group = g
        for l in range(L):
            g = dist.new_group(ranks[l::L], backend=cross_backend)
            if l == self.local_rank:
                self.cross_group = g
        self.cross_on_host = (cross_backend or dist.get_backend(group)) == "gloo"
        self.local = Communicator(group=self.local_group, workspace_bytes=workspace_bytes)
        self._torch = torch
        self._dist = dist

    def _cross_all_reduce(self, t, op: str):
        if self.nodes == 1:
            return t
        dist = self._dist
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
               "prod": dist.ReduceOp.PRODUCT}[op]
        if self.cross_on_host:  # gloo moves host tensors
            h = t.cpu()
            dist.all_reduce(h, op=rop, group=self.cross_group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=rop, group=self.cross_group)
        return t

    def all_reduce(self, tensor, op: str = "sum", out=None, algo: Optional[str] = None):
        """Allreduce ``tensor`` over every rank of every node (in place unless ``out`` is given).
        ops: sum, avg (sum then the 1/world scale), max, min, prod. ``algo`` picks the intra-node
        reduce-scatter / all-gather form ("ring" or the direct exchange). Drop-in for a DDP hook state:
        ``FlexarHookState(communicator=HierarchicalCommunicator())``."""
        torch = self._torch
        dst = tensor if out is None else out
        if out is not None and out.data_ptr() != tensor.data_ptr():
            out.copy_(tensor)
        red = "sum" if op == "avg" else op
        flat = dst.view(-1)
        n = flat.numel()
        m = n // self.L
        main = m * self.L
        if m > 0:
            shard = torch.empty(m, dtype=flat.dtype, device=flat.device)
            self.local.reduce_scatter(flat[:main], shard, op=red, algo=algo)
            self._cross_all_reduce(shard, red)
            self.local.all_gather(shard, flat[:main], algo=algo)
        if main < n:  # fewer than L trailing elements: node allreduce, then across nodes
            tail = flat[main:].clone()
            self.local.all_reduce(tail, op=red)
            self._cross_all_reduce(tail, red)
            flat[main:].copy_(tail)
        if op == "avg":
            flat.mul_(1.0 / self.world)
        return dst

    def close(self):
        self.local.close()
