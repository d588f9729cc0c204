"""Wheel / editable install of the Python package with the native runtime built first.

The gfx950 library (`allreduce_over_mpi_amd/_lib/libflexar.so`, hipcc --offload-arch=gfx950) and the CPython
fast-call module are compiled in-tree by `allreduce_over_mpi_amd/_build.py` before the package is collected, and
ship as package data: `pip wheel . --no-build-isolation` (no index access is needed; setuptools is the only build
dependency). C/C++ users build the same library with CMake (`CMakeLists.txt`).
"""
import os
import sys

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py
from wheel.bdist_wheel import bdist_wheel


class BuildNative(build_py):
    def run(self):
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from allreduce_over_mpi_amd import _build

        _build.build(verbose=True)
        super().run()


class PlatformWheel(bdist_wheel):
    """The wheel carries gfx950 / x86-64 shared objects: a platform wheel, not py3-none-any."""

    def finalize_options(self):
        super().finalize_options()
        self.root_is_pure = False


setup(
    name="allreduce-over-mpi-amd",
    version="0.1.0",
    description="flexar: MI355X-native FlexTree / ring / RHD allreduce (gfx950 HIP executor, xGMI IPC, RCCL transport, "
                "MPI-compatible API, PyTorch c10d backend)",
    packages=find_packages(include=["allreduce_over_mpi_amd", "allreduce_over_mpi_amd.*"]),
    package_data={"allreduce_over_mpi_amd": ["_lib/*.so"]},
    python_requires=">=3.9",
    install_requires=["numpy"],
    extras_require={"torch": ["torch"]},
    cmdclass={"build_py": BuildNative, "bdist_wheel": PlatformWheel},
)
