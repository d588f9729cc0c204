"""In-tree build of the native library ``libflexar.so`` (gfx950 HIP + host C++).

The reference builds one header-only library with CMake + g++/OpenMP
(allreduce_over_mpi/CMakeLists.txt:1-36). Here the runtime is a shared library
with a C ABI: ``csrc/src/*.hip`` are compiled by ``hipcc --offload-arch=gfx950``
and the host-only sources by the host C++ compiler; the result lands in
``allreduce_over_mpi_amd/_lib/`` so it travels with the repo snapshot to the
GPU box. Rebuilds only when a source or header is newer than the library.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
INCLUDE = os.path.join(CSRC, "include")
LIB_DIR = os.path.join(PKG_DIR, "_lib")
LIB_PATH = os.path.join(LIB_DIR, "libflexar.so")
BUILD_DIR = os.path.join(REPO, "build", "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("FLEXAR_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    p = os.path.join(ROCM, "bin", "hipcc")
    return p if os.path.exists(p) else (shutil.which("hipcc") or "hipcc")


def _sources():
    hip = sorted(glob.glob(os.path.join(CSRC, "src", "*.hip")))
    cpp = sorted(glob.glob(os.path.join(CSRC, "src", "*.cpp")))
    return hip, cpp


def _deps():
    return (glob.glob(os.path.join(INCLUDE, "flexar", "*")) + glob.glob(os.path.join(CSRC, "src", "*")))


def needs_build() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(d) > t for d in _deps())


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build step failed:\n  " + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build(verbose: bool = False, force: bool = False) -> str:
    """Compile libflexar.so in-tree; returns its path."""
    if not force and not needs_build():
        return LIB_PATH
    os.makedirs(BUILD_DIR, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    hip, cpp = _sources()
    common = ["-O3", "-fPIC", "-std=c++17", "-I" + INCLUDE, "-Wall", "-Wno-unused-function"]
    jobs = []
    objs = []
    for s in hip:
        o = os.path.join(BUILD_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        jobs.append([_hipcc(), "--offload-arch=" + ARCH, "-munsafe-fp-atomics", *common, "-c", s, "-o", o])
    cxx = os.environ.get("CXX", "g++")
    for s in cpp:
        o = os.path.join(BUILD_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        jobs.append([cxx, *common, "-march=x86-64-v2", "-c", s, "-o", o])
    nproc = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", "8"))))
    with cf.ThreadPoolExecutor(nproc) as ex:
        for out in ex.map(_run, jobs):
            if verbose and out.strip():
                print(out)
    tmp = LIB_PATH + ".tmp"
    _run([_hipcc(), "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp, *objs, "-lpthread"])
    os.replace(tmp, LIB_PATH)
    if verbose:
        print("built", LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    build(verbose=True, force="--force" in sys.argv)
