"""Allreduces captured into one hipGraph, for latency-bound loops.

Tensor-parallel decode issues one small allreduce per layer. Eagerly, every call pays the host launch
path: about 4.4 µs per call on MI355X with the fast-call entry, against a device time of 2.5 µs for a
2-rank LL allreduce (docs/DESIGN.md §13). Captured once and replayed, a call costs
0.4-0.6 µs of host time, so the device floor is what remains.

flexar calls are graph-safe by construction:
- epochs and staging parity live on the device, so no host-side counter is frozen into the graph
  (docs/DESIGN.md §2);
- no allocation or host synchronisation happens on the launch path once a plan exists (the warm-up
  calls below build the plans before capture);
- the copy-engine path (``dma``) bakes a host-side epoch into its copies, so a ``dma`` call (requested
  or selected) is captured as the executor's flat exchange, and once a communicator has been captured
  its eager ``dma`` requests run that exchange too (csrc/src/comm.hip, ``flexar_comm::captured``).

The reference has no counterpart; its allreduce is host-driven MPI (allreduce_over_mpi/mpi_mod.hpp:1167-1221).

    cap = CapturedAllReduce(comm, [a, b, c])      # collective: every rank captures the same sequence
    for step in range(steps):
        a.copy_(x); b.copy_(y); c.copy_(z)        # new inputs into the static buffers
        cap.replay()                              # a, b, c now hold the sums
"""
from __future__ import annotations

from typing import Optional, Sequence, Union


class CapturedAllReduce:
    """A fixed sequence of allreduces on static buffers, captured into one graph.

    ``tensors``: the buffers, reduced in place unless ``outs`` gives an output for each.
    ``algo``: one spec for every call, or a list with one spec per call (None = the selector).
    Construction runs ``warmup`` eager rounds on the same buffers to build every plan, and those rounds
    overwrite the buffers. Fill the inputs after construction. Every rank must construct the same
    sequence and replay it the same number of times, as with any collective.
    """

    def __init__(self, comm, tensors: Sequence, op: str = "sum", outs: Optional[Sequence] = None,
                 algo: Union[None, str, Sequence[Optional[str]]] = None, warmup: int = 1, pool=None):
        import torch

        self.comm = comm
        self.tensors = list(tensors)
        self.outs = list(outs) if outs is not None else [None] * len(self.tensors)
        if len(self.outs) != len(self.tensors):
            raise ValueError("outs must have one entry per tensor")
        algos = list(algo) if isinstance(algo, (list, tuple)) else [algo] * len(self.tensors)
        if len(algos) != len(self.tensors):
            raise ValueError("algo list must have one entry per tensor")
        # the copy-engine path is not replay-safe: capture the executor's flat exchange in its place, and
        # warm up with that same spec so its plan exists before capture (no allocation while capturing)
        self.algos = [self._capturable(t, a) for t, a in zip(self.tensors, algos)]
        self.op = op
        dev = torch.device("cuda", comm.device)
        self.stream = torch.cuda.Stream(device=dev)
        self.stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(self.stream):
            for _ in range(max(1, warmup)):
                self._issue()
        torch.cuda.current_stream(dev).wait_stream(self.stream)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=self.stream, pool=pool):
            self._issue()
        comm.check()

    def _capturable(self, t, algo):
        spec = algo if algo is not None else self.comm.describe(t.numel(), t.dtype).split(" ")[0]
        return "flat+pull" if spec.startswith("dma") else algo

    def _issue(self):
        for t, o, a in zip(self.tensors, self.outs, self.algos):
            self.comm.all_reduce(t, op=self.op, out=o, algo=a)

    def replay(self):
        """Launch every captured allreduce, stream-ordered on the current stream."""
        self.graph.replay()

    @property
    def results(self) -> list:
        return [o if o is not None else t for t, o in zip(self.tensors, self.outs)]
