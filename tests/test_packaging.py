"""The Python package as a wheel (setup.py / pyproject.toml): the native runtime is built first and both shared
objects ship inside a platform wheel; built with no index access (--no-build-isolation)."""
import glob
import os
import shutil
import subprocess
import sys
import zipfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_wheel_carries_the_native_runtime(tmp_path, nv):
    r = subprocess.run([sys.executable, "-m", "pip", "wheel", REPO, "--no-deps", "--no-build-isolation", "-q",
                        "-w", str(tmp_path)], capture_output=True, text=True, timeout=600, cwd=str(tmp_path),
                       env=dict(os.environ, PIP_NO_INDEX="1", PIP_CACHE_DIR=str(tmp_path / "cache")))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    wheels = glob.glob(str(tmp_path / "allreduce_over_mpi_amd-0.1.0-*.whl"))
    assert len(wheels) == 1 and "linux_x86_64" in wheels[0], wheels
    # a platform wheel keeps the package under <name>.data/purelib/ (pip installs it into site-packages)
    names = [n.split("purelib/", 1)[-1] for n in zipfile.ZipFile(wheels[0]).namelist()]
    assert "allreduce_over_mpi_amd/_lib/libflexar.so" in names
    assert any(n.startswith("allreduce_over_mpi_amd/_lib/_fastcall") for n in names)
    assert "allreduce_over_mpi_amd/parallel/backend.py" in names
    # setuptools builds in the source tree: leave it as it was
    for d in ("build/lib", "build/bdist.linux-x86_64", "allreduce_over_mpi_amd.egg-info"):
        shutil.rmtree(os.path.join(REPO, d), ignore_errors=True)
