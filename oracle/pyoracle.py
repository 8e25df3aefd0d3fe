"""ctypes wrapper of the CPU restatement (oracle/cpl_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.  It is the
parity checker and the CPU baseline; the product (centroidalplanner_amd) never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_double, c_int, c_int32, c_int64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libcpl_oracle.so")


def _load():
    if not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    lib = ctypes.CDLL(LIB_PATH)
    IP = POINTER(c_int32)
    DP = POINTER(c_double)
    lib.cplo_dims.argtypes = [c_void_p, IP, IP, IP]
    lib.cplo_dims.restype = c_int
    lib.cplo_structure.argtypes = [c_void_p, IP, IP]
    lib.cplo_structure.restype = c_int
    lib.cplo_bounds.argtypes = [c_void_p, DP, DP, DP, DP]
    lib.cplo_bounds.restype = c_int
    lib.cplo_eval_batch.argtypes = [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_int]
    lib.cplo_eval_batch.restype = c_int
    lib.cplo_time_eval_batch.argtypes = [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_int, c_int]
    lib.cplo_time_eval_batch.restype = c_double
    lib.cplo_max_threads.argtypes = []
    lib.cplo_max_threads.restype = c_int
    return lib


lib = _load()


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def dims(desc):
    n, m, nnz = c_int32(), c_int32(), c_int32()
    st = lib.cplo_dims(ctypes.byref(desc), ctypes.byref(n), ctypes.byref(m), ctypes.byref(nnz))
    if st:
        raise ValueError(f"oracle dims failed: {st}")
    return n.value, m.value, nnz.value


def structure(desc):
    _, _, nnz = dims(desc)
    iRow = np.zeros(nnz, dtype=np.int32)
    jCol = np.zeros(nnz, dtype=np.int32)
    st = lib.cplo_structure(ctypes.byref(desc), iRow.ctypes.data_as(POINTER(c_int32)),
                            jCol.ctypes.data_as(POINTER(c_int32)))
    if st:
        raise ValueError(f"oracle structure failed: {st}")
    return iRow, jCol


def bounds(desc):
    n, m, _ = dims(desc)
    xl, xu, gl, gu = np.zeros(n), np.zeros(n), np.zeros(m), np.zeros(m)
    DP = POINTER(c_double)
    st = lib.cplo_bounds(ctypes.byref(desc), xl.ctypes.data_as(DP), xu.ctypes.data_as(DP), gl.ctypes.data_as(DP),
                         gu.ctypes.data_as(DP))
    if st:
        raise ValueError(f"oracle bounds failed: {st}")
    return xl, xu, gl, gu


def eval_batch(desc, x, mass=None, env_tag=None, outputs=("g", "jac", "f", "grad"), nthreads=None):
    """x: float64 [B, n] host array.  Returns dict of host arrays."""
    n, m, nnz = dims(desc)
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1, n)
    B = x.shape[0]
    mass = None if mass is None else np.ascontiguousarray(mass, dtype=np.float64)
    env_tag = None if env_tag is None else np.ascontiguousarray(env_tag, dtype=np.uint8)
    shapes = {"g": (B, m), "jac": (B, nnz), "f": (B,), "grad": (B, n)}
    out = {k: np.zeros(shapes[k]) for k in outputs}
    if nthreads is None:
        nthreads = lib.cplo_max_threads()
    st = lib.cplo_eval_batch(ctypes.byref(desc), B, _p(x), _p(mass), _p(env_tag), _p(out.get("g")),
                             _p(out.get("jac")), _p(out.get("f")), _p(out.get("grad")), int(nthreads))
    if st:
        raise ValueError(f"oracle eval failed: {st}")
    return out


def time_eval_batch(desc, x, mass=None, env_tag=None, outputs=("g", "jac"), nthreads=1, reps=1):
    """Seconds per batch evaluation (wall clock inside the C library)."""
    n, m, nnz = dims(desc)
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1, n)
    B = x.shape[0]
    shapes = {"g": (B, m), "jac": (B, nnz), "f": (B,), "grad": (B, n)}
    out = {k: np.zeros(shapes[k]) for k in outputs}
    mass = None if mass is None else np.ascontiguousarray(mass, dtype=np.float64)
    env_tag = None if env_tag is None else np.ascontiguousarray(env_tag, dtype=np.uint8)
    t = lib.cplo_time_eval_batch(ctypes.byref(desc), B, _p(x), _p(mass), _p(env_tag), _p(out.get("g")),
                                 _p(out.get("jac")), _p(out.get("f")), _p(out.get("grad")), int(nthreads), int(reps))
    if t < 0:
        raise ValueError("oracle timing failed")
    return t


def max_threads():
    return lib.cplo_max_threads()
