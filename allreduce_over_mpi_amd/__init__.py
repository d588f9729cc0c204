"""allreduce_over_mpi_amd — "flexar", an MI355X-native allreduce framework.

Capabilities of Youhe-Jiang/AllReduce-Over-MPI (FlexTree mixed-radix tree,
ring, FT_TOPO selection, MPI_Allreduce_FT API, benchmark driver, offline cost
model) rebuilt for GPU-resident tensors on MI355X: HIP executor kernels moving
data peer-to-peer over xGMI with fused reductions, a runtime cost-model
selector, torch.distributed integration (ProcessGroup backend, DDP hook).

Layout: ``ops`` (device kernels), ``parallel`` (communicators, backend, DDP
hook), ``utils`` (topology/cost-model helpers, bandwidth math), ``models``
(data-parallel training demo model).
"""
from . import _native  # noqa: F401
from ._native import FlexarError  # noqa: F401

__version__ = "0.1.0"


def native_library_path() -> str:
    return _native.lib_path()


def version() -> str:
    return _native.lib().flexar_version().decode()
