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


def node_size_from_hosts(hosts) -> int:
    """Ranks per node from every rank's hostname: contiguous, equal-sized blocks of ranks per host."""
    world = len(hosts)
    L = hosts.count(hosts[0])
    if world % L or any(hosts[i] != hosts[(i // L) * L] for i in range(world)) or len(set(hosts)) != world // L:
        raise nv.FlexarError(1, "hierarchical allreduce needs contiguous, equal-sized blocks of ranks per host")
    return L


def _node_size(group, world: int) -> int:
    import torch.distributed as dist

    env = int(os.environ.get("FLEXAR_NODE_SIZE", "0") or 0)
    if env > 0:
        return env
    hosts = [None] * world
    dist.all_gather_object(hosts, socket.gethostname(), group=group)
    return node_size_from_hosts(hosts)


class HierarchicalCommunicator:
    """Allreduce over ``group`` (default: WORLD) as intra-node flexar RS -> cross-node allreduce -> AG.

    ``cross_pg``: the cross-node group as a c10d ProcessGroup (the backend builds it from its Store);
    by default it is created with ``torch.distributed.new_group`` (``cross_backend``)."""

    def __init__(self, group=None, node_size: Optional[int] = None, workspace_bytes: int = 0,
                 cross_backend: Optional[str] = None, *, _parts=None):
        import torch
        import torch.distributed as dist

        self._torch = torch
        self._dist = dist
        if _parts is not None:  # from_store()
            (self.rank, self.world, self.L, self.local, self.cross_pg, self.cross_on_host) = _parts
            self.world_size = self.world
            self.nodes = self.world // self.L
            self.local_rank, self.node = self.rank % self.L, self.rank // self.L
            self.group = self.local_group = self.cross_group = None
            return
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
        self.cross_pg = None
        self.cross_on_host = (cross_backend or dist.get_backend(group)) == "gloo"
        self.local = Communicator(group=self.local_group, workspace_bytes=workspace_bytes)

    @classmethod
    def from_store(cls, store, rank: int, world: int, node_size: int, device: int, cross_kind: str = "nccl",
                   workspace_bytes: int = 0, timeout=None):
        """Build from a c10d Store (no torch.distributed default group needed): the node's flexar
        communicator bootstraps through a node-prefixed Store, the cross-node group is a ProcessGroupNCCL
        (RCCL) or ProcessGroupGloo over a prefixed Store, ranked by node index."""
        import datetime

        import torch.distributed as dist

        from .comm import store_exchange

        L = node_size
        if L < 1 or world % L:
            raise nv.FlexarError(1, f"node size {L} does not divide the world size {world}")
        node, lr, nodes = rank // L, rank % L, world // L
        local = Communicator(device=device, rank=lr, world_size=L, workspace_bytes=workspace_bytes,
                             exchange=store_exchange(dist.PrefixStore(f"flexar_node{node}/", store), lr, L, "comm"))
        cstore = dist.PrefixStore(f"flexar_cross{lr}/", store)
        if cross_kind == "gloo":
            cross = dist.ProcessGroupGloo(cstore, node, nodes, timeout or datetime.timedelta(minutes=10))
        else:
            cross = dist.ProcessGroupNCCL(cstore, node, nodes, dist.ProcessGroupNCCL.Options())
        return cls(_parts=(rank, world, L, local, cross, cross_kind == "gloo"))

    def _cross_all_reduce(self, t, op: str):
        if self.nodes == 1:
            return t
        dist = self._dist
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
               "prod": dist.ReduceOp.PRODUCT, "band": dist.ReduceOp.BAND, "bor": dist.ReduceOp.BOR,
               "bxor": dist.ReduceOp.BXOR}[op]
        h = t.cpu() if self.cross_on_host else t  # gloo moves host tensors
        if self.cross_pg is not None:
            o = dist.AllreduceOptions()
            o.reduceOp = rop
            self.cross_pg.allreduce([h], o).wait()
        else:
            dist.all_reduce(h, op=rop, group=self.cross_group)
        if h is not t:
            t.copy_(h)
        return t

    def _cross_gather(self, x):
        """Every node's 1-D ``x`` over the cross-node group, in node order: a [nodes, numel] tensor on x's
        device."""
        dist, torch = self._dist, self._torch
        h = x.cpu() if self.cross_on_host else x
        big = torch.empty((self.nodes, h.numel()), dtype=h.dtype, device=h.device)
        outs = list(big.unbind(0))  # rows of one buffer: the device codec reads them with one stride
        if self.cross_pg is not None:
            self.cross_pg.allgather([outs], [h]).wait()
        else:
            dist.all_gather(outs, h, group=self.cross_group)
        return big.to(x.device)

    def _mx_applies(self, dtype) -> bool:
        """The MX cross-node step runs for fp32 / bf16 / fp16 shards and up to FLEXAR_HIER_MX_MAX_NODES (4)
        nodes: its all-gather moves nodes x 1.03 bytes per element to every node - it grows linearly with the
        node count, where a ring allreduce's 2 (n-1)/n x element bytes does not - so beyond a few nodes the
        exact ring is cheaper. float64 (and every other dtype) takes the exact path."""
        torch = self._torch
        if dtype not in (torch.float32, torch.bfloat16, torch.float16):
            return False
        return self.nodes <= int(os.environ.get("FLEXAR_HIER_MX_MAX_NODES", "4") or 4)

    def _cross_all_reduce_mx(self, t, wire: str, post: float = 1.0):
        """Cross-node SUM of a float shard with OCP MX fp8 on the network (a scale per 32-element block): each
        node's shard is quantised once, payload and scales are all-gathered in one message (1.03 bytes per
        element per node instead of a ring allreduce's 2 (n-1)/n x 4), and every node sums the dequantised
        shards in node order in fp32 - identical results everywhere; ``post`` (AVG's 1 / world) multiplies the
        fp32 sum in the same pass. Worth it for up to ~4 nodes, where the all-gather moves fewer bytes than the
        ring."""
        from ..ops.quant import mx_dequantize, mx_quantize

        torch = self._torch
        if self.nodes == 1:
            if post != 1.0:
                t.copy_((t.float() * post).to(t.dtype))
            return t
        n = t.numel()
        if t.is_cuda:  # native codec (csrc/src/k_mx_codec.hip): one pass to pack, one to dequantise and sum
            from ..ops.quant import mx_pack, mx_unpack_sum

            msgs = self._cross_gather(mx_pack(t.contiguous(), wire))
            if t.dtype == torch.float32 and t.is_contiguous():
                mx_unpack_sum(msgs, n, wire, out=t.view(-1), post=post)
            else:
                t.copy_(mx_unpack_sum(msgs, n, wire, post=post).view(t.shape))
            return t
        q, sb = mx_quantize(t.float(), wire)
        # one message per node: the fp8 payload followed by its scale bytes
        msgs = self._cross_gather(torch.cat([q.view(torch.uint8), sb.to(torch.uint8)]))
        acc = None
        for msg in msgs:
            v = mx_dequantize(msg[:n].view(q.dtype), msg[n:], n)
            acc = v if acc is None else acc + v
        t.copy_((acc * post if post != 1.0 else acc).to(t.dtype))
        return t

    def all_reduce(self, tensor, op: str = "sum", out=None, algo: Optional[str] = None,
                   compress: Optional[str] = None):
        """Allreduce ``tensor`` over every rank of every node (in place unless ``out`` is given).
        ops: sum, avg (sum then the 1/world scale), max, min, prod. ``algo`` picks the intra-node
        reduce-scatter / all-gather form ("ring" or the direct exchange). ``compress="mx_e4m3"`` /
        ``"mx_e5m2"`` (float SUM / AVG): the cross-node step carries OCP MX fp8 (_cross_all_reduce_mx); the
        intra-node steps stay exact. Drop-in for a DDP hook state:
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
        scaled_upto = 0  # elements whose AVG scale is already applied (fused into the MX unpack-sum)
        if m > 0:
            shard = torch.empty(m, dtype=flat.dtype, device=flat.device)
            self.local.reduce_scatter(flat[:main], shard, op=red, algo=algo)
            if compress and red == "sum" and self._mx_applies(flat.dtype):
                # AVG's 1 / world rides in the unpack-sum pass: no separate pass over the
                # shard or over the gathered buffer
                post = 1.0 / self.world if op == "avg" else 1.0
                self._cross_all_reduce_mx(shard, {"mx_e4m3": "e4m3", "mx_e5m2": "e5m2"}[compress], post)
                scaled_upto = main if op == "avg" else 0
            else:
                self._cross_all_reduce(shard, red)
            self.local.all_gather(shard, flat[:main], algo=algo)
        if main < n:  # fewer than L trailing elements: node allreduce, then across nodes
            tail = flat[main:].clone()
            self.local.all_reduce(tail, op=red)
            self._cross_all_reduce(tail, red)
            flat[main:].copy_(tail)
        if op == "avg" and scaled_upto < n:
            flat[scaled_upto:].mul_(1.0 / self.world)
        return dst

    def close(self):
        self.local.close()
