"""C++ host facade (include/cpl/*.hpp, centroidalplanner_amd/host/*.cpp): builds tests/cpp/test_host.cpp
against libcpl_host.so and runs it — API-mirror cases on the CPU, CplTNLP / BatchBroker parity
against the CPU oracle on the GPU."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "centroidalplanner_amd")
OUT = os.path.join(HERE, "_build")
EXE = os.path.join(OUT, "test_host")
SRC = os.path.join(HERE, "cpp", "test_host.cpp")


def _build():
    deps = [SRC, os.path.join(PKG, "libcpl_host.so")] + [
        os.path.join(ROOT, "include", "cpl", h) for h in os.listdir(os.path.join(ROOT, "include", "cpl"))]
    if os.path.exists(EXE) and all(os.path.getmtime(d) <= os.path.getmtime(EXE) for d in deps):
        return EXE
    os.makedirs(OUT, exist_ok=True)
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cmd = ["/opt/rocm/bin/hipcc", "-x", "c++", "-O1", "-std=c++17", "-Wall", "-D__HIP_PLATFORM_AMD__",
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(rocm, "include"), SRC, "-o", EXE + ".tmp",
           "-L" + PKG, "-lcpl_host", "-lcpl_mi355x", "-L" + os.path.join(rocm, "lib"), "-lamdhip64", "-ldl",
           "-Wl,-rpath," + PKG]
    subprocess.run(cmd, check=True)
    os.replace(EXE + ".tmp", EXE)
    return EXE


def _run(args):
    r = subprocess.run([_build()] + args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failed" in r.stdout
    return r.stdout


def test_host_facade_cpu():
    _run([])


@pytest.mark.gpu
def test_host_facade_gpu():
    import pyoracle  # noqa: F401  (builds the oracle library when missing)

    _run(["--gpu", "--oracle", pyoracle.LIB_PATH])
