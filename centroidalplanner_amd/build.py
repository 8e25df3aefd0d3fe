"""In-tree build of the HIP extension (gfx950) and of the oracle checker.

``python -m centroidalplanner_amd.build`` compiles ``csrc/*`` with hipcc into
``centroidalplanner_amd/libcpl_mi355x.so``.  The arithmetic contract needs
``-ffp-contract=off`` (no FMA contraction: the reference's x86-64 build has none) and no
fast-math.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libcpl_mi355x.so")

SOURCES = ["cpl_host.cpp", "cpl_kernels.hip", "cpl_kkt.hip", "cpl_ipm.hip", "cpl_solver.hip", "cpl_check.hip"]
HEADERS = ["cpl_layout.hpp", "cpl_status.hpp", "cpl_wave.hpp", "cpl_accept.hpp", "cpl_kkt_block.hpp", "cpl_kkt_qd.hpp",
           "cpl_kkt_wave.hpp"]

HIPCC_FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-ffp-contract=off",
    "-fno-fast-math",
    "-std=c++17",
    "-fPIC",
    "-shared",
    "-Wall",
    "-Wno-unused-result",
]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP extension cannot be built")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_extension(force: bool = False, verbose: bool = False) -> str:
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "cpl_mi355x.h")]
    if not force and not _stale(LIB, deps):
        return LIB
    cmd = [_hipcc()] + HIPCC_FLAGS + [os.path.join(CSRC, s) for s in SOURCES] + ["-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(LIB + ".tmp", LIB)
    return LIB


HOST_DIR = os.path.join(HERE, "host")
HOST_LIB = os.path.join(HERE, "libcpl_host.so")
HOST_SOURCES = ["cpl_problem.cpp", "cpl_planner.cpp", "cpl_broker.cpp", "cpl_native.cpp"]
HOST_HEADERS = ["Environment.hpp", "CplProblem.hpp", "CentroidalPlanner.hpp", "BatchBroker.hpp"]


def build_host(force: bool = False, verbose: bool = False) -> str:
    """The C++ host facade (cpl::CentroidalPlanner / CoMPlanner / CplProblem / CplTNLP / BatchBroker)
    above the C-ABI: host code only, linked against libcpl_mi355x.so (rpath $ORIGIN)."""
    deps = ([os.path.join(HOST_DIR, s) for s in HOST_SOURCES] +
            [os.path.join(ROOT, "include", "cpl", h) for h in HOST_HEADERS] + [LIB])
    if not force and not _stale(HOST_LIB, deps):
        return HOST_LIB
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cmd = ([_hipcc(), "-x", "c++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-D__HIP_PLATFORM_AMD__",
            "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(rocm, "include")] +
           [os.path.join(HOST_DIR, s) for s in HOST_SOURCES] +
           ["-o", HOST_LIB + ".tmp", "-L" + HERE, "-lcpl_mi355x", "-L" + os.path.join(rocm, "lib"), "-lamdhip64",
            "-Wl,-rpath,$ORIGIN"])
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=HOST_DIR)
    os.replace(HOST_LIB + ".tmp", HOST_LIB)
    return HOST_LIB


def build_oracle(verbose: bool = False) -> str:
    """Build the CPU restatement (test infrastructure) with its own Makefile."""
    odir = os.path.join(ROOT, "oracle")
    cmd = ["make", "-s", "-C", odir]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return os.path.join(odir, "_build", "libcpl_oracle.so")


if __name__ == "__main__":
    print(build_extension(force="--force" in sys.argv, verbose=True))
    print(build_host(force="--force" in sys.argv, verbose=True))
