"""ctypes binding of oracle/_build/liboracle.so — CPU ORACLE (test infrastructure only).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
See oracle/pdeinv_oracle.c for what each function restates and the parity status.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

POT = {"quadratic": 0, "gmm": 1, "meanfield": 2, "none": 3}


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH) or (
        os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "pdeinv_oracle.c"))
    ):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        i64, i32, u32, u64, f32 = (ctypes.c_int64, ctypes.c_int, ctypes.c_uint32,
                                   ctypes.c_uint64, ctypes.c_float)
        _lib.oracle_philox4x32_10.argtypes = [P, P, P]
        _lib.oracle_sde_simulate.argtypes = [i64, i64, i32, i32, f32, f32, f32, i32, u64, u32,
                                             i32, i32, f32, P, i32, P, P, P, i64, P, P, P]
        _lib.oracle_sde_simulate.restype = ctypes.c_int
        _lib.oracle_moments.argtypes = [P, i64, i32, i64, P]
        _lib.oracle_gaussian_sample.argtypes = [i64, i32, u64, u32, i64, P, P, P]
        _lib.oracle_philox_fill.argtypes = [u64, u32, u32, i64, P]
        _lib.oracle_sim_normals.argtypes = [u64, u64, u32, i32, P]
        _lib.oracle_shift_u.argtypes = [u64, u64, u32]
        _lib.oracle_shift_u.restype = f32
        _lib.oracle_gmm_grad.argtypes = [i32, i32, f32, P, P, P, P]
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def philox(ctr, key):
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().oracle_philox4x32_10(_p(c), _p(k), _p(out))
    return out


def philox_fill(seed, ctr_z, ctr_w, n_blocks):
    out = np.zeros((n_blocks, 4), dtype=np.uint32)
    lib().oracle_philox_fill(seed, ctr_z, ctr_w, n_blocks, _p(out))
    return out


def sim_normals(seed, particle, ctr_z, d):
    out = np.zeros(d, dtype=np.float32)
    lib().oracle_sim_normals(seed, particle, ctr_z, d, _p(out))
    return out


def sde_simulate(z0, n_steps, dt, gamma, kind="quadratic", params=None, n_centers=0, sigma=1.0,
                 has_center=False, seed=0, counter_offset=0, particle_offset=0,
                 noise_scale=float(np.sqrt(2.0)), random_shift=True, noise=None, shift_u=None,
                 outputs=("last", "traj", "tau")):
    """Returns dict with last [N,2d], traj [n,N,2d] (time-major), tau [n,N] (fp32)."""
    z0 = np.ascontiguousarray(z0, dtype=np.float32)
    N, m = z0.shape
    d = m // 2
    params = np.ascontiguousarray(np.zeros(1) if params is None else params, dtype=np.float32).ravel()
    noise = None if noise is None else np.ascontiguousarray(noise, dtype=np.float32)
    shift_u = None if shift_u is None else np.ascontiguousarray(shift_u, dtype=np.float32)
    out = {}
    last = np.zeros((N, m), np.float32) if "last" in outputs else None
    traj = np.zeros((n_steps, N, m), np.float32) if "traj" in outputs else None
    tau = np.zeros((n_steps, N), np.float32) if "tau" in outputs else None
    rc = lib().oracle_sde_simulate(N, particle_offset, d, n_steps, dt, gamma, noise_scale,
                                   int(random_shift), seed, counter_offset, POT[kind], n_centers,
                                   sigma, _p(params), int(has_center), _p(noise), _p(shift_u),
                                   _p(z0), m, _p(traj), _p(tau), _p(last))
    if rc != 0:
        raise RuntimeError(f"oracle_sde_simulate failed: {rc}")
    for k, v in (("last", last), ("traj", traj), ("tau", tau)):
        if v is not None:
            out[k] = v
    return out


def moments(z):
    z = np.ascontiguousarray(z, dtype=np.float32)
    z2 = z.reshape(-1, z.shape[-1])
    m = z2.shape[1]
    out = np.zeros(1 + m + m * (m + 1) // 2, np.float64)
    lib().oracle_moments(_p(z2), z2.shape[0], m, m, _p(out))
    return out


def gaussian_sample(n, mean, cov_half, seed, counter_offset=0, row_offset=0):
    mean = np.ascontiguousarray(mean, dtype=np.float32)
    cov_half = np.ascontiguousarray(cov_half, dtype=np.float32)
    m = mean.shape[0]
    out = np.zeros((n, m), np.float32)
    lib().oracle_gaussian_sample(n, m, seed, counter_offset, row_offset, _p(mean), _p(cov_half), _p(out))
    return out


def gmm_grad(x, mus, sigma=1.0):
    x = np.ascontiguousarray(x, dtype=np.float32)
    mus = np.ascontiguousarray(mus, dtype=np.float32)
    K, d = mus.shape
    g = np.zeros_like(x)
    v = np.zeros(x.shape[0], np.float32)
    for i in range(x.shape[0]):
        val = ctypes.c_float(0.0)
        lib().oracle_gmm_grad(d, K, sigma, _p(mus), _p(x[i]), _p(g[i]), ctypes.byref(val))
        v[i] = val.value
    return v, g
