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
LIB_DIR = os.environ.get("FLEXAR_LIB_DIR") or os.path.join(PKG_DIR, "_lib")
LIB_PATH = os.path.join(LIB_DIR, "libflexar.so")
BUILD_DIR = os.path.join(REPO, "build", "obj" + os.environ.get("FLEXAR_BUILD_TAG", ""))
EXTRA_CFLAGS = os.environ.get("FLEXAR_EXTRA_CFLAGS", "").split()
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


def _fastcall_paths():
    import sysconfig

    src = os.path.join(CSRC, "python", "fastcall.c")
    out = os.path.join(LIB_DIR, "_fastcall" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
    return src, out


FASTCALL_PATH = _fastcall_paths()[1]


def _fastcall_stale() -> bool:
    src, out = _fastcall_paths()
    return not os.path.exists(out) or os.path.getmtime(src) > os.path.getmtime(out)


def needs_build() -> bool:
    if not os.path.exists(LIB_PATH) or _fastcall_stale():
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(d) > t for d in _deps())


def build_fastcall(verbose: bool = False) -> str:
    """The CPython fast-call module (csrc/python/fastcall.c): plain C against the Python headers, no
    link against libflexar.so (it receives the entry points' addresses at import)."""
    import sysconfig

    src, out = _fastcall_paths()
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = out + ".tmp"
    _run([os.environ.get("CC", "gcc"), "-O2", "-shared", "-fPIC", "-Wall", "-I" + sysconfig.get_paths()["include"],
          src, "-o", tmp])
    os.replace(tmp, out)
    if verbose:
        print("built", out)
    return out


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build step failed:\n  " + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build(verbose: bool = False, force: bool = False) -> str:
    """Compile libflexar.so (and the fast-call module) in-tree; returns the library's path."""
    if force or _fastcall_stale():
        build_fastcall(verbose)
    if not force and not needs_build():
        return LIB_PATH
    os.makedirs(BUILD_DIR, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    hip, cpp = _sources()
    common = ["-O3", "-fPIC", "-std=c++17", "-I" + INCLUDE, "-Wall", "-Wno-unused-function"]
    jobs = []
    objs = []

    def stale(src, obj):
        # an object is rebuilt when its source or a header it included (compiler -MMD list) is newer
        dep = obj + ".d"
        if force or not os.path.exists(obj) or not os.path.exists(dep):
            return True
        t = os.path.getmtime(obj)
        with open(dep) as f:
            files = f.read().replace("\\\n", " ").split(":", 1)[-1].split()
        return any(not os.path.exists(x) or os.path.getmtime(x) > t for x in [src] + files)

    for s in hip:
        o = os.path.join(BUILD_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        if stale(s, o):
            jobs.append([_hipcc(), "--offload-arch=" + ARCH, "-munsafe-fp-atomics", *common, *EXTRA_CFLAGS, "-MMD", "-MF",
                         o + ".d", "-c", s, "-o", o])
    cxx = os.environ.get("CXX", "g++")
    for s in cpp:
        o = os.path.join(BUILD_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        if stale(s, o):
            jobs.append([cxx, *common, "-march=x86-64-v2", "-MMD", "-MF", o + ".d", "-c", s, "-o", o])
    # objects of sources that no longer exist must not be linked
    objs = [o for o in objs if o]
    nproc = max(1, min(max(1, len(jobs)), int(os.environ.get("MAX_JOBS", "8"))))
    # the slowest translation units first: the typed executors dominate the build
    jobs.sort(key=lambda j: 0 if "k_mx" in j[-3] else 1)
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


BIN_DIR = os.path.join(REPO, "bin")
MPI_HOME = os.environ.get("FLEXAR_MPI_HOME", "/opt/conda")
TOOLS = {
    # name: (sources, needs MPI, needs RCCL)
    "flexar_bench": (["bench/flexar_bench.cpp"], True, True),
    "test_mpi_allreduce": (["tests/cpp/test_mpi_allreduce.cpp"], True, False),
    "flexar_plan": (["tools/flexar_plan.cpp"], False, False),
}


def mpi_available() -> bool:
    return os.path.exists(os.path.join(MPI_HOME, "include", "mpi.h")) and \
        os.path.exists(os.path.join(MPI_HOME, "lib", "libmpi.so.12"))


def _mpi_libdir() -> str:
    """A private dir with only the MPI runtime libs (MPI_HOME/lib also ships an old libstdc++)."""
    d = os.path.join(BIN_DIR, "mpilib")
    os.makedirs(d, exist_ok=True)
    for name in ("libmpi.so.12", "libgfortran.so.4", "libquadmath.so.0"):
        src = os.path.join(MPI_HOME, "lib", name)
        dst = os.path.join(d, name)
        if os.path.exists(src) and not os.path.lexists(dst):
            os.symlink(src, dst)
    return d


def git_version() -> str:
    try:
        return subprocess.run(["git", "-C", REPO, "describe", "--always", "--dirty"], stdout=subprocess.PIPE,
                              stderr=subprocess.DEVNULL, text=True).stdout.strip() or "unknown"
    except Exception:
        return "unknown"


def build_tools(names=None, verbose: bool = False):
    """Build the C++ executables (benchmark driver, MPI test harness, planner CLI) into bin/."""
    lib = build(verbose=verbose)
    os.makedirs(BIN_DIR, exist_ok=True)
    names = names or list(TOOLS)
    built = {}
    jobs = []
    for name in names:
        srcs, need_mpi, need_rccl = TOOLS[name]
        if need_mpi and not mpi_available():
            continue
        out = os.path.join(BIN_DIR, name)
        srcp = [os.path.join(REPO, x) for x in srcs]
        deps = srcp + _deps()
        if os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps) and \
                os.path.getmtime(lib) <= os.path.getmtime(out):
            built[name] = out
            continue
        # host-only C++ (HIP runtime API + MPI): the plain host compiler, linked against libamdhip64
        cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__",
               "-I" + os.path.join(ROCM, "include"), "-I" + INCLUDE, "-DFLEXAR_GIT_VERSION=\"%s\"" % git_version(), *srcp,
               "-o", out, "-L" + LIB_DIR, "-lflexar", "-Wl,-rpath,$ORIGIN/../allreduce_over_mpi_amd/_lib", "-L" + os.path.join(ROCM, "lib"),
               "-lamdhip64", "-Wl,-rpath," + os.path.join(ROCM, "lib"), "-lpthread"]
        if need_mpi:
            cmd.insert(5, "-I" + os.path.join(MPI_HOME, "include"))
            d = _mpi_libdir()
            cmd += [os.path.join(d, "libmpi.so.12"), "-Wl,-rpath,$ORIGIN/mpilib", "-Wl,-rpath-link," + d]
        if need_rccl:
            cmd += ["-L" + os.path.join(ROCM, "lib"), "-lrccl"]
        jobs.append((name, out, cmd))
    with cf.ThreadPoolExecutor(max(1, min(len(jobs), 4))) as ex:
        for (name, out, _), res in zip(jobs, ex.map(lambda j: _run(j[2]), jobs)):
            built[name] = out
    return built


if __name__ == "__main__":
    build(verbose=True, force="--force" in sys.argv)
    if "--tools" in sys.argv:
        print(build_tools(verbose=True))
