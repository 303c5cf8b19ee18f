"""ctypes binding of libpdeinv.so (the C ABI in include/pdeinv.h).

This is the only door from the Python mirror of the reference into the hot path. It fails
loudly: if the library is missing, or a call is made without a GPU, it raises — there is no
CPU fallback anywhere in the product path. Error codes map to the
reference's exception types: INVALID -> ValueError, UNSUPPORTED -> NotImplementedError,
HIP -> RuntimeError.

PyTorch-ROCm is plumbing here: it owns device memory (caching allocator) and streams; every
pointer handed to the library is a torch tensor's data_ptr() on the current stream. torch is
imported before the library is dlopen'ed so that both share torch's libamdhip64.so.7.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from typing import Optional

import numpy as np
import torch

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC_DIR = os.path.join(_PKG_DIR, "csrc")
LIB_PATH = os.path.join(_PKG_DIR, "_build", "libpdeinv.so")

PDEINV_OK, PDEINV_ERR_INVALID, PDEINV_ERR_UNSUPPORTED, PDEINV_ERR_HIP = 0, -1, -2, -3
POT_QUADRATIC, POT_GMM, POT_MEANFIELD_QUADRATIC, POT_NONE = 0, 1, 2, 3
MAX_DIM, MAX_PARAMS = 16, 256
KFP_NOUT = 9
KFP_SLOTS = ("loss", "loss ground truth", "grad_norm", "loss_nabla", "loss_Hessian",
             "loss_friction", "loss_nabla_true", "loss_initial", "loss_terminal")
GMM_NACC = 8
# PDEINV_GMM_ACC_* slot names (include/pdeinv.h), shared by the GMM and MLP residual accumulators
GMM_ACC_SLOTS = ("loss", "loss_gt", "nabla", "hessian", "friction", "nabla_true", "initial", "terminal")
SQRT2 = math.sqrt(2.0)

ABI_VERSION = 10  # PDEINV_ABI_VERSION of include/pdeinv.h this binding was written against

# Every exported symbol of include/pdeinv.h (tests check the library exports all of them).
EXPORTED_SYMBOLS = (
    "pdeinv_moment_len", "pdeinv_sde_workspace_bytes", "pdeinv_sde_simulate",
    "pdeinv_sde_simulate_mf_kmv_workspace_bytes", "pdeinv_sde_simulate_mf_kmv",
    "pdeinv_mf_workspace_bytes", "pdeinv_mf_step", "pdeinv_sde_tau0",
    "pdeinv_moments_workspace_bytes", "pdeinv_moments", "pdeinv_residual_kfp_quadratic",
    "pdeinv_residual_kfp_gmm_workspace_bytes", "pdeinv_residual_kfp_gmm",
    "pdeinv_residual_kfp_gmm_finalize", "pdeinv_gmm_potential", "pdeinv_gaussian_sample",
    "pdeinv_gaussian_sample_grouped", "pdeinv_fp_rows", "pdeinv_fp_exact_sample",
    "pdeinv_philox_fill", "pdeinv_gather_subsample", "pdeinv_abi_version", "pdeinv_last_error",
    "pdeinv_runtime_version", "pdeinv_moments_batched_workspace_bytes", "pdeinv_moments_batched",
    "pdeinv_kmv_weights_workspace_bytes", "pdeinv_kmv_weights", "pdeinv_residual_kmv",
    "pdeinv_residual_kmv_workspace_bytes",
    "pdeinv_mlp_param_count", "pdeinv_rocblas_calls", "pdeinv_residual_kfp_mlp_workspace_bytes", "pdeinv_residual_kfp_mlp",
    "pdeinv_kfp_terms_finalize", "pdeinv_gather_random_step", "pdeinv_mlp_fused_supported",
    "pdeinv_adam_update", "pdeinv_realnvp_param_count", "pdeinv_realnvp_logdensity",
    "pdeinv_realnvp_grad_workspace", "pdeinv_realnvp_value_and_grad",
    "pdeinv_residual_kmv_mlp_workspace_bytes", "pdeinv_residual_kmv_mlp", "pdeinv_kmv_mlp_path",
    "pdeinv_mf_sums_len", "pdeinv_mf_sums_workspace_bytes", "pdeinv_mf_sums", "pdeinv_mf_mean_path",
    "pdeinv_kmv_moments_weights_workspace_bytes", "pdeinv_kmv_moments_weights",
    "pdeinv_kmv_moments_weights_mf_sums_workspace_bytes", "pdeinv_kmv_moments_weights_mf_sums",
    "pdeinv_sde_simulate_kfp_gmm_workspace_bytes", "pdeinv_sde_simulate_kfp_gmm",
    "pdeinv_sde_simulate_mf_next_workspace_bytes", "pdeinv_sde_simulate_mf_next", "pdeinv_ou_exact_sample",
)


class PotentialDesc(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("n_centers", ctypes.c_int32), ("sigma", ctypes.c_float),
                ("has_center", ctypes.c_int32), ("params", ctypes.c_void_p)]


class SdeDesc(ctypes.Structure):
    _fields_ = [("n_particles", ctypes.c_int64), ("particle_offset", ctypes.c_int64),
                ("dim", ctypes.c_int32), ("n_steps", ctypes.c_int32), ("dt", ctypes.c_float),
                ("gamma", ctypes.c_float), ("noise_scale", ctypes.c_float),
                ("random_shift", ctypes.c_int32), ("seed", ctypes.c_uint64),
                ("counter_offset", ctypes.c_uint32), ("ld_z0", ctypes.c_int64),
                ("potential", PotentialDesc), ("d_noise", ctypes.c_void_p),
                ("d_shift_u", ctypes.c_void_p), ("d_meanfield", ctypes.c_void_p)]


class KfpQuadDesc(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int32), ("gamma", ctypes.c_float), ("total_time", ctypes.c_float),
                ("tilde_F", ctypes.c_void_p)]


class KmvDesc(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int32), ("n_sets", ctypes.c_int32), ("gamma", ctypes.c_float),
                ("tilde_F", ctypes.c_void_p)]


class KfpMlpDesc(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int32), ("n_layers", ctypes.c_int32), ("width", ctypes.c_int32),
                ("out_features", ctypes.c_int32), ("true_kind", ctypes.c_int32), ("n_centers_true", ctypes.c_int32),
                ("sigma_true", ctypes.c_float), ("true_params", ctypes.c_void_p), ("gamma", ctypes.c_float),
                ("c_nabla", ctypes.c_float), ("c_hess", ctypes.c_float), ("c_fric", ctypes.c_float),
                ("c_true", ctypes.c_float), ("c_init", ctypes.c_float), ("c_term", ctypes.c_float),
                ("chunk_rows", ctypes.c_int64), ("impl", ctypes.c_int32), ("boundary_value", ctypes.c_int32)]


class OuDesc(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("taylor_degree", ctypes.c_int32), ("squarings", ctypes.c_int32),
                ("t_min", ctypes.c_double), ("t_max", ctypes.c_double), ("d_powers", ctypes.c_void_p),
                ("d_m0", ctypes.c_void_p), ("d_P0", ctypes.c_void_p)]


class KmvMlpDesc(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int32), ("n_layers", ctypes.c_int32), ("width", ctypes.c_int32),
                ("out_features", ctypes.c_int32), ("n_sets", ctypes.c_int32), ("n_rows", ctypes.c_int64),
                ("gamma", ctypes.c_float), ("tilde_F", ctypes.c_void_p), ("chunk_rows", ctypes.c_int64),
                ("impl", ctypes.c_int32)]


MLP_IMPL_AUTO, MLP_IMPL_LIBRARY, MLP_IMPL_FUSED, MLP_IMPL_PAIRS_RING = 0, 1, 2, 3  # PAIRS_RING: kmv_mlp only

ACTIVATIONS = {"celu": 0, "relu": 1, "tanh": 2, "elu": 3, "silu": 4, "softplus": 5, "gelu": 6}


class RealNvpDesc(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int32), ("n_layers", ctypes.c_int32), ("embed_time_dim", ctypes.c_int32),
                ("ignore_time", ctypes.c_int32), ("soft_init", ctypes.c_float), ("activation", ctypes.c_int32),
                ("masks", ctypes.c_void_p), ("base_mean", ctypes.c_void_p), ("base_inv_cov", ctypes.c_void_p),
                ("base_log_det", ctypes.c_float)]


class KfpGmmDesc(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int32), ("n_centers", ctypes.c_int32), ("sigma", ctypes.c_float),
                ("n_centers_true", ctypes.c_int32), ("sigma_true", ctypes.c_float),
                ("mus_true", ctypes.c_void_p), ("gamma", ctypes.c_float),
                ("c_nabla", ctypes.c_float), ("c_hess", ctypes.c_float), ("c_fric", ctypes.c_float),
                ("c_true", ctypes.c_float), ("c_init", ctypes.c_float), ("c_term", ctypes.c_float)]


_lib = None


def build(force: bool = False, jobs: int = 8) -> str:
    """Compile libpdeinv.so in-tree (hipcc --offload-arch=gfx950)."""
    args = ["make", "-C", CSRC_DIR, f"-j{jobs}"]
    if force:
        subprocess.check_call(["make", "-C", CSRC_DIR, "clean"])
    subprocess.check_call(args)
    return LIB_PATH


def lib():
    """The loaded library; raises if it was not built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("PDEINV_LIBRARY", LIB_PATH)  # A/B timing of alternative builds (tools/)
    if not os.path.exists(path):
        raise RuntimeError(f"pdeinv native library missing at {path}; run __graft_entry__.build() "
                           "(the hot path has no CPU fallback)")
    L = ctypes.CDLL(path)
    P, i32, i64, u32, u64, f32 = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32,
                                  ctypes.c_uint64, ctypes.c_float)
    sig = {
        "pdeinv_moment_len": (i32, [i32]),
        "pdeinv_sde_workspace_bytes": (ctypes.c_size_t, [P]),
        "pdeinv_sde_simulate": (i32, [P, P, P, P, P, P, P, P]),
        "pdeinv_mf_workspace_bytes": (ctypes.c_size_t, [P]),
        "pdeinv_mf_step": (i32, [P, i32, P, P, P, P, P, P, P, P]),
        "pdeinv_sde_tau0": (i32, [P, P, P]),
        "pdeinv_sde_simulate_kfp_gmm_workspace_bytes": (ctypes.c_size_t, [P, P]),
        "pdeinv_sde_simulate_kfp_gmm": (i32, [P, P, P, P, P, P, P, P, P, P]),
        "pdeinv_mf_sums_len": (i64, [P]),
        "pdeinv_mf_sums_workspace_bytes": (ctypes.c_size_t, [P]),
        "pdeinv_sde_simulate_mf_next_workspace_bytes": (ctypes.c_size_t, [P]),
        "pdeinv_sde_simulate_mf_next": (i32, [P, P, P, P, P, P, P, P, P, P]),
        "pdeinv_sde_simulate_mf_kmv_workspace_bytes": (ctypes.c_size_t, [P, i32]),
        "pdeinv_sde_simulate_mf_kmv": (i32, [P, P, P, P, P, f32, P, P, P, P, P, P, P, P]),
        "pdeinv_mf_sums": (i32, [P, P, P, P, P]),
        "pdeinv_mf_mean_path": (i32, [P, P, P, P, P]),
        "pdeinv_kmv_moments_weights_workspace_bytes": (ctypes.c_size_t, [i64, i64, i32]),
        "pdeinv_kmv_moments_weights": (i32, [i32, f32, P, P, i64, i64, i64, i64, P, P, P, P]),
        "pdeinv_kmv_moments_weights_mf_sums_workspace_bytes": (ctypes.c_size_t, [i64, i64, i32, P]),
        "pdeinv_kmv_moments_weights_mf_sums": (i32, [i32, f32, P, P, i64, i64, i64, i64, P, P, P, P, P, P, P]),
        "pdeinv_moments_workspace_bytes": (ctypes.c_size_t, [i64, i32]),
        "pdeinv_moments": (i32, [P, i64, i32, i64, P, P, P]),
        "pdeinv_residual_kfp_quadratic": (i32, [P, P, P, P, P, P]),
        "pdeinv_residual_kfp_gmm_workspace_bytes": (ctypes.c_size_t, [P, i64, i64, i64]),
        "pdeinv_residual_kfp_gmm": (i32, [P, P, i64, i64, P, i64, i64, P, i64, i64, P, P, P, P]),
        "pdeinv_residual_kfp_gmm_finalize": (i32, [P, P, P, P, P]),
        "pdeinv_gmm_potential": (i32, [i32, i32, f32, P, P, i64, i64, P, P, P]),
        "pdeinv_gaussian_sample": (i32, [i64, i32, u64, u32, i64, P, P, P, P]),
        "pdeinv_gaussian_sample_grouped": (i32, [i64, i64, i32, u64, u32, i64, P, P, P, P]),
        "pdeinv_ou_exact_sample": (i32, [P, i64, i64, u64, u32, u32, i64, P, P, P, P, P, P]),
        "pdeinv_philox_fill": (i32, [u64, u32, u32, i64, P, P]),
        "pdeinv_gather_subsample": (i32, [P, i64, i32, i32, P, i64, P, i32, P, P]),
        "pdeinv_abi_version": (i32, []),
        "pdeinv_last_error": (ctypes.c_char_p, []),
        "pdeinv_runtime_version": (i32, []),
        "pdeinv_moments_batched_workspace_bytes": (ctypes.c_size_t, [i64, i64, i32]),
        "pdeinv_moments_batched": (i32, [P, i64, i64, i32, i64, i64, P, P, P]),
        "pdeinv_kmv_weights_workspace_bytes": (ctypes.c_size_t, [i64, i64, i32]),
        "pdeinv_kmv_weights": (i32, [i32, f32, P, P, i64, i64, i64, i64, P, P, P, P]),
        "pdeinv_residual_kmv_workspace_bytes": (ctypes.c_size_t, [P]),
        "pdeinv_residual_kmv": (i32, [P, P, P, P, P, P, P, P]),
        "pdeinv_mlp_param_count": (i64, [i32, i32, i32, i32]),
        "pdeinv_rocblas_calls": (i64, []),
        "pdeinv_mlp_fused_supported": (i32, [i32, i32, i32, i32]),
        "pdeinv_adam_update": (i32, [P, P, P, P, i64, f32, f32, f32, f32, f32, i32, P]),
        "pdeinv_realnvp_param_count": (i64, [P]),
        "pdeinv_realnvp_logdensity": (i32, [P, P, P, i64, P, i64, i64, P, P]),
        "pdeinv_realnvp_grad_workspace": (i64, [P, i64]),
        "pdeinv_realnvp_value_and_grad": (i32, [P, P, P, i64, P, i64, i64, P, P, P, i64, P]),
        "pdeinv_residual_kfp_mlp_workspace_bytes": (ctypes.c_size_t, [P]),
        "pdeinv_residual_kfp_mlp": (i32, [P, P, i64, i64, P, i64, i64, P, i64, i64, P, P, P, P, P]),
        "pdeinv_kfp_terms_finalize": (i32, [P, P, i64, f32, P, P]),
        "pdeinv_residual_kmv_mlp_workspace_bytes": (ctypes.c_size_t, [P]),
        "pdeinv_kmv_mlp_path": (ctypes.c_int, [P]),
        "pdeinv_residual_kmv_mlp": (i32, [P, P, i64, i64, P, P, P, P, P, P]),
        "pdeinv_gather_random_step": (i32, [P, i64, i32, i32, u64, u32, P, P, P]),
        "pdeinv_fp_rows": (i32, [P, i64, i64, i32, i32, P, P]),
        "pdeinv_fp_exact_sample": (i32, [i64, i32, u64, u32, i64, f32, f32, P, P, P, P, P, P, P, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.pdeinv_abi_version() != ABI_VERSION:
        raise RuntimeError("libpdeinv ABI version mismatch")
    _lib = L
    return _lib


def _check(rc: int, what: str) -> None:
    if rc == PDEINV_OK:
        return
    msg = f"{what}: {lib().pdeinv_last_error().decode(errors='replace')}"
    if rc == PDEINV_ERR_INVALID:
        raise ValueError(msg)
    if rc == PDEINV_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise RuntimeError(msg)


def _require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("pdeinv hot path needs a ROCm GPU (no CPU fallback)")


def _dev(t: Optional[torch.Tensor], name: str, dtype=torch.float32) -> Optional[ctypes.c_void_p]:
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    return ctypes.c_void_p(t.data_ptr())


def _rows(t: torch.Tensor, name: str, m: int):
    """A 2-D [n, m] view with unit inner stride; returns (ptr, n, ld)."""
    if t.dim() != 2 or t.shape[1] != m:
        raise ValueError(f"{name} must have shape [n, {m}], got {tuple(t.shape)}")
    if t.shape[0] > 0 and t.stride(1) != 1:
        raise ValueError(f"{name} must have unit stride along its last axis")
    return _dev(t, name), t.shape[0], (t.stride(0) if t.shape[0] > 1 else m)


def stream_handle() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def moment_len(m: int) -> int:
    return 1 + m + m * (m + 1) // 2


def _host_f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32).ravel())


# -----------------------------------------------------------------------------------------
# simulator
# -----------------------------------------------------------------------------------------
def make_potential(kind: int, params=None, n_centers: int = 0, sigma: float = 1.0,
                   has_center: bool = False):
    host = _host_f32(np.zeros(1) if params is None else params)
    desc = PotentialDesc(kind, int(n_centers), float(sigma), int(has_center),
                         host.ctypes.data_as(ctypes.c_void_p))
    return desc, host  # keep `host` alive while desc is used


def _sim_desc(z0: torch.Tensor, n_steps: int, dt: float, gamma: float, potential: dict, seed: int,
              counter_offset: int, particle_offset: int, noise_scale: float, random_shift: bool,
              noise: Optional[torch.Tensor], shift_u: Optional[torch.Tensor]):
    """(SdeDesc, keep-alive host params, z0 pointer) for the simulator entry points."""
    if z0.dim() != 2 or z0.shape[1] % 2:
        raise ValueError("q0_p0 must be [N, 2d]")
    N, m = z0.shape
    d = m // 2
    p_desc, p_host = make_potential(**potential)
    desc = SdeDesc()
    desc.n_particles = N
    desc.particle_offset = int(particle_offset)
    desc.dim = d
    desc.n_steps = int(n_steps)
    desc.dt = float(dt)
    desc.gamma = float(gamma)
    desc.noise_scale = float(noise_scale)
    desc.random_shift = int(bool(random_shift))
    desc.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    desc.counter_offset = int(counter_offset) & 0xFFFFFFFF
    z0p, _, ld = _rows(z0, "q0_p0", m) if N > 0 else (None, 0, m)
    desc.ld_z0 = ld
    desc.potential = p_desc
    if noise is not None:
        if tuple(noise.shape) != (n_steps + 1, N, d) or not noise.is_contiguous():
            raise ValueError(f"noise must be contiguous [{n_steps + 1}, {N}, {d}]")
        desc.d_noise = _dev(noise, "noise")
    if shift_u is not None:
        if tuple(shift_u.shape) != (N,) or not shift_u.is_contiguous():
            raise ValueError(f"shift_u must be contiguous [{N}]")
        desc.d_shift_u = _dev(shift_u, "shift_u")
    return desc, p_host, z0p


def _sim_outputs(res: dict, z0: torch.Tensor, n_steps: int, traj: bool, tau: bool, last: bool) -> dict:
    N, m = z0.shape
    dev = z0.device
    if traj and "traj" not in res:
        res["traj"] = torch.empty((n_steps, N, m), device=dev, dtype=torch.float32)
    if tau and "tau" not in res:
        res["tau"] = torch.empty((n_steps, N), device=dev, dtype=torch.float32)
    if last and "last" not in res:
        res["last"] = torch.empty((N, m), device=dev, dtype=torch.float32)
    return res


def sde_simulate(z0: torch.Tensor, n_steps: int, dt: float, gamma: float, potential: dict, *,
                 seed: int, counter_offset: int = 0, particle_offset: int = 0,
                 noise_scale: float = SQRT2, random_shift: bool = True,
                 noise: Optional[torch.Tensor] = None, shift_u: Optional[torch.Tensor] = None,
                 traj: bool = True, tau: bool = True, last: bool = True,
                 moments: bool = False, out: Optional[dict] = None) -> dict:
    """utils/sampling_utils.py:25-52 on the GPU. Returns time-major traj [n, N, 2d]."""
    _require_gpu()
    desc, p_host, z0p = _sim_desc(z0, n_steps, dt, gamma, potential, seed, counter_offset, particle_offset,
                                  noise_scale, random_shift, noise, shift_u)
    m = z0.shape[1]
    res = _sim_outputs({} if out is None else out, z0, n_steps, traj, tau, last)
    ws = None
    if moments:
        if "moments" not in res:
            res["moments"] = torch.empty((3, moment_len(m)), device=z0.device, dtype=torch.float64)
        nbytes = lib().pdeinv_sde_workspace_bytes(ctypes.byref(desc))
        ws = torch.empty(max(nbytes // 4, 1), device=z0.device, dtype=torch.float32)
    rc = lib().pdeinv_sde_simulate(
        ctypes.byref(desc), z0p, _dev(res.get("traj") if traj else None, "traj"),
        _dev(res.get("tau") if tau else None, "tau"), _dev(res.get("last") if last else None, "last"),
        _dev(ws, "workspace"), _dev(res.get("moments") if moments else None, "moments", torch.float64),
        stream_handle())
    del p_host
    _check(rc, "pdeinv_sde_simulate")
    return res


def sde_simulate_kfp_gmm(z0: torch.Tensor, n_steps: int, dt: float, gamma: float, potential: dict, res_desc,
                         mus: torch.Tensor, *, seed: int, counter_offset: int = 0, particle_offset: int = 0,
                         noise_scale: float = SQRT2, random_shift: bool = True, noise: Optional[torch.Tensor] = None,
                         shift_u: Optional[torch.Tensor] = None, traj: bool = True, tau: bool = True,
                         last: bool = True, out: Optional[dict] = None) -> dict:
    """The GMM simulator with the KFP residual of a GMM model fused in (pdeinv_sde_simulate_kfp_gmm):
    initial = z0, 0T = every trajectory row, terminal = last; the trajectory is never re-read. res_desc
    from kfp_gmm_desc(..., n_init=N_global, n_term=N_global, n_0T=N_global * n_steps) whose true GMM is
    the simulated potential. Returns the simulator outputs plus "acc" (fp64 [8 + K d], the
    residual_kfp_gmm accumulator: all-reduce, then residual_kfp_gmm_finalize)."""
    _require_gpu()
    desc, p_host, z0p = _sim_desc(z0, n_steps, dt, gamma, potential, seed, counter_offset, particle_offset,
                                  noise_scale, random_shift, noise, shift_u)
    rdesc, _keep = res_desc
    K, d = rdesc.n_centers, rdesc.dim
    if tuple(mus.shape) != (K, d):
        raise ValueError(f"mus must be [{K}, {d}]")
    mus_c = mus.contiguous()
    res = _sim_outputs({} if out is None else out, z0, n_steps, traj, tau, last)
    nbytes = lib().pdeinv_sde_simulate_kfp_gmm_workspace_bytes(ctypes.byref(desc), ctypes.byref(rdesc))
    ws = torch.empty(max(nbytes // 4, 1), device=z0.device, dtype=torch.float32)
    res["acc"] = torch.empty(GMM_NACC + K * d, device=z0.device, dtype=torch.float64)
    rc = lib().pdeinv_sde_simulate_kfp_gmm(
        ctypes.byref(desc), ctypes.byref(rdesc), _dev(mus_c, "mus"), z0p,
        _dev(res.get("traj") if traj else None, "traj"), _dev(res.get("tau") if tau else None, "tau"),
        _dev(res.get("last") if last else None, "last"), _dev(ws, "workspace"), _dev(res["acc"], "acc", torch.float64),
        stream_handle())
    del p_host
    _check(rc, "pdeinv_sde_simulate_kfp_gmm")
    return res


def sde_tau0(N: int, dt: float, *, seed: int, counter_offset: int = 0, particle_offset: int = 0,
             random_shift: bool = True, device="cuda") -> torch.Tensor:
    _require_gpu()
    desc = SdeDesc()
    desc.n_particles = N
    desc.particle_offset = particle_offset
    desc.dim = 1
    desc.n_steps = 1
    desc.dt = dt
    desc.noise_scale = SQRT2
    desc.random_shift = int(random_shift)
    desc.seed = seed
    desc.counter_offset = counter_offset
    desc.potential = PotentialDesc(POT_NONE, 0, 1.0, 0, None)
    out = torch.empty(N, device=device, dtype=torch.float32)
    _check(lib().pdeinv_sde_tau0(ctypes.byref(desc), _dev(out, "tau0"), stream_handle()), "pdeinv_sde_tau0")
    return out


def mf_sums(desc: SdeDesc, z0: torch.Tensor) -> torch.Tensor:
    """Rank-local [count, sum x0, sum v0, sum_i xi_{i,s} (s = 0..n)] fp64 of the McKean–Vlasov
    ensemble (pdeinv_mf_sums) — all-reduce(sum) it, then mf_mean_path."""
    _require_gpu()
    L = int(lib().pdeinv_mf_sums_len(ctypes.byref(desc)))
    if L <= 0:
        raise ValueError("mf_sums: bad descriptor")
    if z0.dim() != 2 or z0.shape[0] != desc.n_particles or z0.shape[1] != 2 * desc.dim:
        raise ValueError(f"mf_sums: z0 must be [{desc.n_particles}, {2 * desc.dim}]")
    if z0.shape[0] and z0.stride(1) != 1:
        raise ValueError("mf_sums: z0 must have unit inner stride")
    desc.ld_z0 = z0.stride(0) if z0.shape[0] > 1 else 2 * desc.dim
    ws = torch.empty(max(int(lib().pdeinv_mf_sums_workspace_bytes(ctypes.byref(desc))) // 4, 1), device=z0.device,
                     dtype=torch.float32)
    out = torch.empty(L, device=z0.device, dtype=torch.float64)
    _check(lib().pdeinv_mf_sums(ctypes.byref(desc), _dev(z0, "z0") if z0.shape[0] else None, _dev(ws, "ws"),
                                _dev(out, "sums", torch.float64), stream_handle()), "pdeinv_mf_sums")
    return out


def mf_mean_path(desc: SdeDesc, sums: torch.Tensor, xsum: bool = True):
    """(xbar [n+1, d] fp32, xsum [n+2, 1+d] fp64 or None) from the all-reduced mf_sums."""
    _require_gpu()
    n, d = desc.n_steps, desc.dim
    xbar = torch.empty((n + 1, d), device=sums.device, dtype=torch.float32)
    xs = torch.empty((n + 2, 1 + d), device=sums.device, dtype=torch.float64) if xsum else None
    _check(lib().pdeinv_mf_mean_path(ctypes.byref(desc), _dev(sums, "sums", torch.float64), _dev(xbar, "xbar"),
                                     _dev(xs, "xsum", torch.float64), stream_handle()), "pdeinv_mf_mean_path")
    return xbar, xs


def sde_simulate_desc(desc: SdeDesc, z0: torch.Tensor, traj: Optional[torch.Tensor], tau: Optional[torch.Tensor],
                      last: Optional[torch.Tensor]) -> None:
    """pdeinv_sde_simulate with a prepared descriptor (the McKean–Vlasov fused path: desc.d_meanfield
    set to mf_mean_path's xbar). Outputs are caller-allocated (time-major traj [n, N, 2d])."""
    _require_gpu()
    N, m, n = desc.n_particles, 2 * desc.dim, desc.n_steps
    for t, shape, name in ((traj, (n, N, m), "traj"), (tau, (n, N), "tau"), (last, (N, m), "last")):
        if t is not None and (tuple(t.shape) != shape or not t.is_contiguous()):
            raise ValueError(f"{name} must be contiguous {shape}")
    if N and (z0.dim() != 2 or tuple(z0.shape) != (N, m) or z0.stride(1) != 1):
        raise ValueError(f"z0 must be [{N}, {m}] with unit inner stride")
    desc.ld_z0 = z0.stride(0) if N > 1 else m
    _check(lib().pdeinv_sde_simulate(ctypes.byref(desc), _dev(z0, "z0") if N else None, _dev(traj, "traj"),
                                     _dev(tau, "tau"), _dev(last, "last"), None, None, stream_handle()),
           "pdeinv_sde_simulate")


def sde_simulate_mf_next(desc: SdeDesc, z0: torch.Tensor, traj: torch.Tensor, tau: Optional[torch.Tensor],
                         last: torch.Tensor, next_desc: SdeDesc, z0_next: torch.Tensor) -> torch.Tensor:
    """sde_simulate_desc (fused McKean-Vlasov path) that also returns the NEXT simulate's rank-local mf_sums
    (pdeinv_sde_simulate_mf_next: the noise sums drawn inside the simulator). next_desc differs from desc in
    counter_offset only."""
    _require_gpu()
    N, m, n = desc.n_particles, 2 * desc.dim, desc.n_steps
    for t, shape, name in ((traj, (n, N, m), "traj"), (tau, (n, N), "tau"), (last, (N, m), "last")):
        if t is not None and (tuple(t.shape) != shape or not t.is_contiguous()):
            raise ValueError(f"{name} must be contiguous {shape}")
    for t, name in ((z0, "z0"), (z0_next, "z0_next")):
        if N and (t.dim() != 2 or tuple(t.shape) != (N, m) or t.stride(1) != 1):
            raise ValueError(f"{name} must be [{N}, {m}] with unit inner stride")
    desc.ld_z0 = z0.stride(0) if N > 1 else m
    next_desc.ld_z0 = z0_next.stride(0) if N > 1 else m
    nbytes = int(lib().pdeinv_sde_simulate_mf_next_workspace_bytes(ctypes.byref(desc)))
    ws = torch.empty(max((nbytes + 3) // 4, 1), device=z0.device, dtype=torch.float32)
    sums = torch.empty(int(lib().pdeinv_mf_sums_len(ctypes.byref(next_desc))), device=z0.device, dtype=torch.float64)
    _check(lib().pdeinv_sde_simulate_mf_next(ctypes.byref(desc), _dev(z0, "z0") if N else None, _dev(traj, "traj"),
                                             _dev(tau, "tau"), _dev(last, "last"), ctypes.byref(next_desc),
                                             _dev(z0_next, "z0_next") if N else None, _dev(ws, "ws"),
                                             _dev(sums, "sums_next", torch.float64), stream_handle()),
           "pdeinv_sde_simulate_mf_next")
    return sums


def sde_simulate_mf_kmv(desc: SdeDesc, z0: torch.Tensor, traj: Optional[torch.Tensor], tau: Optional[torch.Tensor],
                        last: torch.Tensor, gamma: float, coef: torch.Tensor, next_desc: Optional[SdeDesc] = None,
                        z0_next: Optional[torch.Tensor] = None):
    """sde_simulate_desc (fused McKean-Vlasov path) that also forms the quadratic-Phi KMV residual's per-stamp
    sums of its own trajectory rows — (mom [n, moment_len(2d)], wst [n, moment_len(d)]) fp64, rank-local, what
    kmv_moments_weights(d, gamma, coef, traj, n, N, N * 2d, 2d) returns up to the fp32 summation order — without
    reading the trajectory back (traj may be None). With next_desc (counter offset differs only) also the next
    simulate's rank-local mf_sums: (mom, wst, sums_next). pdeinv_sde_simulate_mf_kmv."""
    _require_gpu()
    N, m, n, d = desc.n_particles, 2 * desc.dim, desc.n_steps, desc.dim
    for t, shape, name in ((traj, (n, N, m), "traj"), (tau, (n, N), "tau"), (last, (N, m), "last")):
        if t is not None and (tuple(t.shape) != shape or not t.is_contiguous()):
            raise ValueError(f"{name} must be contiguous {shape}")
    if tuple(coef.shape) != (n, kmv_ncoef(d)) or not coef.is_contiguous():
        raise ValueError(f"coef must be contiguous [{n}, {kmv_ncoef(d)}]")
    if N and (z0.dim() != 2 or tuple(z0.shape) != (N, m) or z0.stride(1) != 1):
        raise ValueError(f"z0 must be [{N}, {m}] with unit inner stride")
    desc.ld_z0 = z0.stride(0) if N > 1 else m
    if next_desc is not None:
        if z0_next is None or (N and (z0_next.dim() != 2 or tuple(z0_next.shape) != (N, m) or z0_next.stride(1) != 1)):
            raise ValueError(f"z0_next must be [{N}, {m}] with unit inner stride")
        next_desc.ld_z0 = z0_next.stride(0) if N > 1 else m
    nbytes = int(lib().pdeinv_sde_simulate_mf_kmv_workspace_bytes(ctypes.byref(desc), int(next_desc is not None)))
    ws = torch.empty(max((nbytes + 3) // 4, 1), device=z0.device, dtype=torch.float32)
    mom = torch.empty((n, moment_len(m)), device=z0.device, dtype=torch.float64)
    wst = torch.empty((n, moment_len(d)), device=z0.device, dtype=torch.float64)
    sums = (torch.empty(int(lib().pdeinv_mf_sums_len(ctypes.byref(next_desc))), device=z0.device, dtype=torch.float64)
            if next_desc is not None else None)
    _check(lib().pdeinv_sde_simulate_mf_kmv(ctypes.byref(desc), _dev(z0, "z0") if N else None, _dev(traj, "traj"),
                                            _dev(tau, "tau"), _dev(last, "last"), float(gamma), _dev(coef, "coef"),
                                            _dev(mom, "mom", torch.float64), _dev(wst, "wst", torch.float64),
                                            ctypes.byref(next_desc) if next_desc is not None else None,
                                            _dev(z0_next, "z0_next") if (next_desc is not None and N) else None,
                                            _dev(sums, "sums_next", torch.float64), _dev(ws, "ws"), stream_handle()),
           "pdeinv_sde_simulate_mf_kmv")
    return (mom, wst) if next_desc is None else (mom, wst, sums)


def mf_step(desc: SdeDesc, s: int, z: torch.Tensor, z_out: torch.Tensor, tau_row, xbar_sum: torch.Tensor,
            ws: torch.Tensor, xsum_out: torch.Tensor) -> None:
    rc = lib().pdeinv_mf_step(ctypes.byref(desc), int(s), _dev(z, "z"), _dev(z_out, "z_out"),
                              _dev(tau_row, "tau_row"), None, _dev(xbar_sum, "xbar_sum", torch.float64),
                              _dev(ws, "workspace"), _dev(xsum_out, "xsum", torch.float64), stream_handle())
    _check(rc, "pdeinv_mf_step")


# -----------------------------------------------------------------------------------------
# moments + residuals
# -----------------------------------------------------------------------------------------
def moments(z: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[count, sum z, sum z_i z_j (i<=j)] fp64 of the rows of z ([..., m], inner stride 1)."""
    _require_gpu()
    m = z.shape[-1]
    z2 = z.reshape(-1, m)
    ptr, n, ld = _rows(z2, "z", m) if z2.shape[0] > 0 else (None, 0, m)
    if out is None:
        out = torch.empty(moment_len(m), device=z.device, dtype=torch.float64)
    nbytes = lib().pdeinv_moments_workspace_bytes(n, m)
    if nbytes == 0:
        raise NotImplementedError(f"moments: m={m} unsupported (1..16)")
    ws = torch.empty(nbytes // 4, device=z.device, dtype=torch.float32)
    _check(lib().pdeinv_moments(ptr, n, m, ld, _dev(ws, "ws"), _dev(out, "out", torch.float64),
                                stream_handle()), "pdeinv_moments")
    return out


def residual_kfp_quadratic(mom3: torch.Tensor, theta_flat: torch.Tensor, tilde_F, gamma: float,
                           total_time: float):
    """kinetic_fokker_planck.py:11-69 for V_theta = x.(xK+b); returns (out[9], grad_flat)."""
    _require_gpu()
    d = int(round(math.sqrt(theta_flat.numel() + 0.25) - 0.5))
    if d * d + d != theta_flat.numel():
        raise ValueError("theta must hold d*d + d values")
    if tuple(mom3.shape) != (3, moment_len(2 * d)) or not mom3.is_contiguous():
        raise ValueError("moments must be contiguous [3, moment_len(2d)] fp64")
    F = _host_f32(tilde_F)
    desc = KfpQuadDesc(d, float(gamma), float(total_time), F.ctypes.data_as(ctypes.c_void_p))
    out = torch.empty(KFP_NOUT, device=mom3.device, dtype=torch.float32)
    grad = torch.empty_like(theta_flat)
    theta_c = theta_flat.contiguous()  # bound to a name: alive until the launch has been issued
    _check(lib().pdeinv_residual_kfp_quadratic(ctypes.byref(desc), _dev(mom3, "moments", torch.float64),
                                               _dev(theta_c, "theta"), _dev(out, "out"),
                                               _dev(grad, "grad"), stream_handle()),
           "pdeinv_residual_kfp_quadratic")
    return out, grad


def kfp_gmm_desc(dim, n_centers, mus_true, gamma, total_time, n_init, n_term, n_0T, sigma=1.0,
                 sigma_true=1.0, world_scale=1.0):
    """Descriptor with the reference's loss weights (kinetic_fokker_planck.py:33-50).
    world_scale = 1/world_size turns per-rank sums into the pmap mean (trainer.py:52)."""
    mt = _host_f32(mus_true)
    M = float(n_0T)
    c = dict(c_nabla=1.0 / M, c_hess=-2.0 / M, c_fric=2.0 * gamma / M, c_true=1.0 / M,
             c_init=(-2.0 / (total_time * n_init)) if n_init else 0.0,
             c_term=(2.0 / (total_time * n_term)) if n_term else 0.0)
    c = {k: v * world_scale for k, v in c.items()}
    desc = KfpGmmDesc(int(dim), int(n_centers), float(sigma), int(mt.size // dim), float(sigma_true),
                      mt.ctypes.data_as(ctypes.c_void_p), float(gamma), c["c_nabla"], c["c_hess"],
                      c["c_fric"], c["c_true"], c["c_init"], c["c_term"])
    return desc, mt


def residual_kfp_gmm(desc_keep, z_init: torch.Tensor, z_term: torch.Tensor, z_0T: torch.Tensor,
                     mus: torch.Tensor) -> torch.Tensor:
    """Fused per-sample GMM residual + adjoint -> fp64 accumulator [8 + K*d]."""
    _require_gpu()
    desc, _keep = desc_keep
    d, K = desc.dim, desc.n_centers
    m = 2 * d
    pi, ni, ldi = _rows(z_init, "initial", m) if z_init.shape[0] else (None, 0, m)
    pt, nt, ldt = _rows(z_term, "terminal", m) if z_term.shape[0] else (None, 0, m)
    p0, n0, ld0 = _rows(z_0T, "0T", m)
    if tuple(mus.shape) != (K, d):
        raise ValueError(f"mus must be [{K}, {d}]")
    nbytes = lib().pdeinv_residual_kfp_gmm_workspace_bytes(ctypes.byref(desc), ni, nt, n0)
    ws = torch.empty(max(nbytes // 4, 1), device=z_0T.device, dtype=torch.float32)
    acc = torch.empty(GMM_NACC + K * d, device=z_0T.device, dtype=torch.float64)
    mus_c = mus.contiguous()
    rc = lib().pdeinv_residual_kfp_gmm(ctypes.byref(desc), pi, ni, ldi, pt, nt, ldt, p0, n0, ld0,
                                       _dev(mus_c, "mus"), _dev(ws, "ws"),
                                       _dev(acc, "acc", torch.float64), stream_handle())
    _check(rc, "pdeinv_residual_kfp_gmm")
    return acc


def residual_kfp_gmm_finalize(desc_keep, acc: torch.Tensor):
    desc, _keep = desc_keep
    out = torch.empty(KFP_NOUT, device=acc.device, dtype=torch.float32)
    grad = torch.empty(desc.n_centers * desc.dim, device=acc.device, dtype=torch.float32)
    _check(lib().pdeinv_residual_kfp_gmm_finalize(ctypes.byref(desc), _dev(acc, "acc", torch.float64),
                                                  _dev(out, "out"), _dev(grad, "grad"), stream_handle()),
           "pdeinv_residual_kfp_gmm_finalize")
    return out, grad.view(desc.n_centers, desc.dim)


# -----------------------------------------------------------------------------------------
# potentials, samplers, streams
# -----------------------------------------------------------------------------------------
def gmm_potential(x: torch.Tensor, mus, sigma: float = 1.0, value: bool = True, grad: bool = True):
    _require_gpu()
    mh = np.asarray(mus, dtype=np.float32)
    K, d = mh.shape
    ptr, n, ld = _rows(x, "x", d) if x.shape[0] else (None, 0, d)
    v = torch.empty(n, device=x.device, dtype=torch.float32) if value else None
    g = torch.empty((n, d), device=x.device, dtype=torch.float32) if grad else None
    mh = _host_f32(mh)
    _check(lib().pdeinv_gmm_potential(d, K, float(sigma), mh.ctypes.data_as(ctypes.c_void_p), ptr, n, ld,
                                      _dev(v, "value"), _dev(g, "grad"), stream_handle()),
           "pdeinv_gmm_potential")
    return v, g


def gaussian_sample(n: int, mean: torch.Tensor, cov_half: torch.Tensor, *, seed: int,
                    counter_offset: int = 0, row_offset: int = 0) -> torch.Tensor:
    _require_gpu()
    m = mean.shape[0]
    out = torch.empty((n, m), device=mean.device, dtype=torch.float32)
    mean_c, cov_c = mean.contiguous(), cov_half.contiguous()
    _check(lib().pdeinv_gaussian_sample(int(n), int(m), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                        int(counter_offset) & 0xFFFFFFFF, int(row_offset),
                                        _dev(mean_c, "mean"), _dev(cov_c, "cov_half"),
                                        _dev(out, "out"), stream_handle()), "pdeinv_gaussian_sample")
    return out


def gaussian_sample_grouped(rows_per_group: int, means: torch.Tensor, cov_halves: torch.Tensor, *, seed: int,
                            counter_offset: int = 0, row_offset: int = 0) -> torch.Tensor:
    """[G * rows_per_group, m]: rows of group g drawn from N(means[g], cov_halves[g] cov_halves[g]^T)."""
    _require_gpu()
    G, m = means.shape
    if cov_halves.shape != (G, m, m):
        raise ValueError(f"cov_halves must be [{G}, {m}, {m}], got {tuple(cov_halves.shape)}")
    out = torch.empty((G * int(rows_per_group), m), device=means.device, dtype=torch.float32)
    means_c, covs_c = means.contiguous(), cov_halves.contiguous()
    _check(lib().pdeinv_gaussian_sample_grouped(int(G), int(rows_per_group), int(m), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                                int(counter_offset) & 0xFFFFFFFF, int(row_offset),
                                                _dev(means_c, "means"),
                                                _dev(covs_c, "cov_halves"), _dev(out, "out"),
                                                stream_handle()), "pdeinv_gaussian_sample_grouped")
    return out


class OuExactSampler:
    """The exact kinetic-OU sampler on the device (pdeinv_ou_exact_sample; …_OU.py:140-156): groups of rows, group g
    from N(m(t_g), P(t_g)) at t_g ~ U(t_min, t_max) drawn on the device. `powers` = B^0..B^K of the Van Loan block
    B = [[-F, L], [0, F^T]] (host fp64, once per problem), `squarings` s with |B|_1 t_max / 2^s <= 1."""

    def __init__(self, powers: np.ndarray, squarings: int, m0: np.ndarray, P0: np.ndarray, t_min: float, t_max: float,
                 device="cuda"):
        _require_gpu()
        K1, n2, _ = powers.shape
        self.n = n2 // 2
        self._pw = torch.as_tensor(np.ascontiguousarray(powers), dtype=torch.float64, device=device)
        self._m0 = torch.as_tensor(np.ascontiguousarray(m0, dtype=np.float64), device=device)
        self._P0 = torch.as_tensor(np.ascontiguousarray(P0, dtype=np.float64), device=device)
        self.desc = OuDesc(self.n, K1 - 1, int(squarings), float(t_min), float(t_max), self._pw.data_ptr(),
                           self._m0.data_ptr(), self._P0.data_ptr())
        self.device = device

    def sample(self, n_groups: int, rows_per_group: int, *, seed: int, ctr_t: int = 0, ctr_z: int = 0,
               row_offset: int = 0, t: torch.Tensor = None, want_moments: bool = False):
        """rows [n_groups * rows_per_group, n]; with want_moments also (t [G], means [G, n], factors [G, n, n])."""
        G, n = int(n_groups), self.n
        out = torch.empty((G * int(rows_per_group), n), device=self.device, dtype=torch.float32)
        extra = None
        if want_moments:
            extra = (torch.empty(G, device=self.device), torch.empty((G, n), device=self.device),
                     torch.empty((G, n, n), device=self.device))
        if t is not None and (t.dtype != torch.float32 or t.numel() != G or not t.is_contiguous()):
            raise ValueError(f"t must be a contiguous float32 [{G}] tensor")
        ptr = (lambda x: x.data_ptr() if x is not None else None)
        _check(lib().pdeinv_ou_exact_sample(ctypes.byref(self.desc), G, int(rows_per_group),
                                            int(seed) & 0xFFFFFFFFFFFFFFFF, int(ctr_t) & 0xFFFFFFFF,
                                            int(ctr_z) & 0xFFFFFFFF, int(row_offset), ptr(t),
                                            *(ptr(x) for x in (extra or (None, None, None))), out.data_ptr(),
                                            stream_handle()), "pdeinv_ou_exact_sample")
        return (out, *extra) if want_moments else out


def philox_fill(seed: int, ctr_z: int, ctr_w: int, n_blocks: int, device="cuda") -> torch.Tensor:
    _require_gpu()
    out = torch.empty((n_blocks, 4), device=device, dtype=torch.int32)
    _check(lib().pdeinv_philox_fill(seed, ctr_z, ctr_w, n_blocks, _dev(out, "out", torch.int32),
                                    stream_handle()), "pdeinv_philox_fill")
    return out


def gather_subsample(traj_tm: torch.Tensor, traj_idx: torch.Tensor, time_idx: torch.Tensor) -> torch.Tensor:
    """consistency.py:97-118 gather from a time-major [n, N, m] trajectory -> [n_sel*n_t, m]."""
    _require_gpu()
    n, N, m = traj_tm.shape
    if not traj_tm.is_contiguous():
        raise ValueError("trajectory must be contiguous time-major [n, N, m]")
    ti = traj_idx.to(torch.int32).contiguous()
    si = time_idx.to(torch.int32).contiguous()
    out = torch.empty((ti.numel() * si.numel(), m), device=traj_tm.device, dtype=torch.float32)
    _check(lib().pdeinv_gather_subsample(_dev(traj_tm, "traj"), N, n, m, _dev(ti, "traj_idx", torch.int32),
                                         ti.numel(), _dev(si, "time_idx", torch.int32), si.numel(),
                                         _dev(out, "out"), stream_handle()), "pdeinv_gather_subsample")
    return out


# -----------------------------------------------------------------------------------------
# McKean–Vlasov residual path
# -----------------------------------------------------------------------------------------
def kmv_ncoef(d: int) -> int:
    return 3 * d + 2 + 2 * d * d


def _set_view(z: torch.Tensor, n_sets: int, n_rows: int, set_stride: int, ld: int, width: int):
    if z.dtype != torch.float32 or not z.is_cuda:
        raise ValueError("samples must be fp32 device tensors")
    if z.stride(-1) != 1:
        raise ValueError("samples must have unit inner stride")
    need = (n_sets - 1) * set_stride + (n_rows - 1) * ld + width if n_rows > 0 else 0
    avail = z.untyped_storage().nbytes() // 4 - z.storage_offset()
    if need > avail:  # checked on the host: the kernel trusts these strides
        raise ValueError("set/row strides run past the end of the sample buffer")


def moments_batched(z: torch.Tensor, n_sets: int, n_rows: int, m: int, set_stride: int, ld: int) -> torch.Tensor:
    """[n_sets, moment_len(m)] fp64: set t = rows z[t*set_stride + r*ld : +m] (floats)."""
    _require_gpu()
    _set_view(z, n_sets, n_rows, set_stride, ld, m)
    nbytes = lib().pdeinv_moments_batched_workspace_bytes(n_sets, n_rows, m)
    if nbytes == 0:
        raise NotImplementedError(f"moments_batched: m={m} unsupported")
    ws = torch.empty(nbytes // 4, device=z.device, dtype=torch.float32)
    out = torch.empty((n_sets, moment_len(m)), device=z.device, dtype=torch.float64)
    _check(lib().pdeinv_moments_batched(_dev(z, "z"), n_sets, n_rows, m, set_stride, ld, _dev(ws, "ws"),
                                        _dev(out, "out", torch.float64), stream_handle()), "pdeinv_moments_batched")
    return out


def kmv_weights(d: int, gamma: float, coef: torch.Tensor, z: torch.Tensor, n_sets: int, n_rows: int,
                set_stride: int, ld: int, want_ds: bool = False):
    """Per time stamp [sum c, sum c x, sum c x x^T] fp64 (c = ds2 + ds^2 + gamma ds) and optionally
    the per-particle (ds log rho, ds2 log rho) [n_sets, n_rows, 2]."""
    _require_gpu()
    if tuple(coef.shape) != (n_sets, kmv_ncoef(d)) or not coef.is_contiguous():
        raise ValueError(f"coef must be contiguous [{n_sets}, {kmv_ncoef(d)}]")
    _set_view(z, n_sets, n_rows, set_stride, ld, d)
    nbytes = lib().pdeinv_kmv_weights_workspace_bytes(n_sets, n_rows, d)
    ws = torch.empty(max(nbytes // 4, 1), device=z.device, dtype=torch.float32)
    out = torch.empty((n_sets, moment_len(d)), device=z.device, dtype=torch.float64)
    ds = torch.empty((n_sets, n_rows, 2), device=z.device, dtype=torch.float32) if want_ds else None
    _check(lib().pdeinv_kmv_weights(d, float(gamma), _dev(coef, "coef"), _dev(z, "z"), n_sets, n_rows, set_stride,
                                    ld, _dev(ds, "ds"), _dev(ws, "ws"), _dev(out, "out", torch.float64),
                                    stream_handle()), "pdeinv_kmv_weights")
    return out, ds


def kmv_moments_weights(d: int, gamma: float, coef: torch.Tensor, z: torch.Tensor, n_sets: int, n_rows: int,
                        set_stride: int, ld: int):
    """moments_batched(m = 2d) and kmv_weights in one read of the rows: (mom [n_sets, moment_len(2d)],
    wst [n_sets, moment_len(d)]) fp64 (pdeinv_kmv_moments_weights)."""
    _require_gpu()
    if tuple(coef.shape) != (n_sets, kmv_ncoef(d)) or not coef.is_contiguous():
        raise ValueError(f"coef must be contiguous [{n_sets}, {kmv_ncoef(d)}]")
    _set_view(z, n_sets, n_rows, set_stride, ld, 2 * d)
    nbytes = lib().pdeinv_kmv_moments_weights_workspace_bytes(n_sets, n_rows, d)
    if nbytes == 0:
        raise NotImplementedError(f"kmv_moments_weights: dim={d} unsupported (1..8)")
    ws = torch.empty((nbytes + 3) // 4, device=z.device, dtype=torch.float32)
    mom = torch.empty((n_sets, moment_len(2 * d)), device=z.device, dtype=torch.float64)
    wst = torch.empty((n_sets, moment_len(d)), device=z.device, dtype=torch.float64)
    _check(lib().pdeinv_kmv_moments_weights(d, float(gamma), _dev(coef, "coef"), _dev(z, "z"), n_sets, n_rows,
                                            set_stride, ld, _dev(ws, "ws"), _dev(mom, "mom", torch.float64),
                                            _dev(wst, "wst", torch.float64), stream_handle()),
           "pdeinv_kmv_moments_weights")
    return mom, wst


def kmv_moments_weights_mf_sums(d: int, gamma: float, coef: torch.Tensor, z: torch.Tensor, n_sets: int, n_rows: int,
                                set_stride: int, ld: int, next_desc: SdeDesc, z0_next: torch.Tensor):
    """kmv_moments_weights fused with the NEXT McKean-Vlasov simulate's mf_sums (the steady state of the KMV
    loop): (mom, wst, sums_next) — sums_next equals mf_sums(next_desc, z0_next) up to the fp32 partial-sum
    order (pdeinv_kmv_moments_weights_mf_sums)."""
    _require_gpu()
    if tuple(coef.shape) != (n_sets, kmv_ncoef(d)) or not coef.is_contiguous():
        raise ValueError(f"coef must be contiguous [{n_sets}, {kmv_ncoef(d)}]")
    _set_view(z, n_sets, n_rows, set_stride, ld, 2 * d)
    if z0_next.dim() != 2 or z0_next.shape[0] != next_desc.n_particles or z0_next.shape[1] != 2 * d or \
            z0_next.stride(1) != 1:
        raise ValueError(f"z0_next must be [{next_desc.n_particles}, {2 * d}] with unit inner stride")
    next_desc.ld_z0 = z0_next.stride(0) if z0_next.shape[0] > 1 else 2 * d
    nbytes = lib().pdeinv_kmv_moments_weights_mf_sums_workspace_bytes(n_sets, n_rows, d, ctypes.byref(next_desc))
    if nbytes == 0:
        raise NotImplementedError(f"kmv_moments_weights_mf_sums: dim={d} unsupported (1..8)")
    ws = torch.empty((nbytes + 3) // 4, device=z.device, dtype=torch.float32)
    mom = torch.empty((n_sets, moment_len(2 * d)), device=z.device, dtype=torch.float64)
    wst = torch.empty((n_sets, moment_len(d)), device=z.device, dtype=torch.float64)
    sums = torch.empty(int(lib().pdeinv_mf_sums_len(ctypes.byref(next_desc))), device=z.device, dtype=torch.float64)
    _check(lib().pdeinv_kmv_moments_weights_mf_sums(d, float(gamma), _dev(coef, "coef"), _dev(z, "z"), n_sets, n_rows,
                                                    set_stride, ld, _dev(ws, "ws"), _dev(mom, "mom", torch.float64),
                                                    _dev(wst, "wst", torch.float64), ctypes.byref(next_desc),
                                                    _dev(z0_next, "z0_next"), _dev(sums, "sums", torch.float64),
                                                    stream_handle()),
           "pdeinv_kmv_moments_weights_mf_sums")
    return mom, wst, sums


def residual_kmv_mlp(dims, params_flat: torch.Tensor, z: torch.Tensor, n_sets: int, n_rows: int, set_stride: int,
                     ld: int, ds: torch.Tensor, tilde_F, gamma: float, chunk_rows: int = 1 << 18,
                     impl: int = MLP_IMPL_AUTO):
    """kinetic_mckean_vlasov.py:11-120 for Phi_theta = V_hypothesis over every pair of each time
    stamp's particles (pdeinv_residual_kmv_mlp). ds = (ds log rho, ds2 log rho) [n_sets, n_rows, 2]
    from kmv_weights(want_ds=True). Returns (acc fp64 [8], grad fp32 [P]) — finalize with
    kfp_terms_finalize(acc, grad, 1.0)."""
    _require_gpu()
    d, W, O = dims[0], dims[1], dims[-1]
    L = len(dims) - 2
    if L < 1 or any(w != W for w in dims[1:-1]):
        raise NotImplementedError("KMV MLP residual: hidden layers must share one width (V_hypothesis)")
    P = lib().pdeinv_mlp_param_count(d, L, W, O)
    if params_flat.numel() != P or not params_flat.is_contiguous():
        raise ValueError(f"KMV MLP residual: params must be a contiguous flat vector of {P} floats")
    _set_view(z, n_sets, n_rows, set_stride, ld, 2 * d)
    if tuple(ds.shape) != (n_sets, n_rows, 2) or not ds.is_contiguous():
        raise ValueError(f"KMV MLP residual: ds must be contiguous [{n_sets}, {n_rows}, 2]")
    F = _host_f32(tilde_F)
    desc = KmvMlpDesc(d, L, W, O, int(n_sets), int(n_rows), float(gamma), F.ctypes.data_as(ctypes.c_void_p),
                      int(chunk_rows), int(impl))
    nbytes = lib().pdeinv_residual_kmv_mlp_workspace_bytes(ctypes.byref(desc))
    ws = torch.empty(nbytes // 4, device=z.device, dtype=torch.float32)
    acc = torch.zeros(GMM_NACC, device=z.device, dtype=torch.float64)
    grad = torch.zeros(P, device=z.device, dtype=torch.float32)
    _check(lib().pdeinv_residual_kmv_mlp(ctypes.byref(desc), _dev(z, "z"), int(set_stride), int(ld), _dev(ds, "ds"),
                                         _dev(params_flat, "params"), _dev(ws, "ws"),
                                         _dev(acc, "acc", torch.float64), _dev(grad, "grad"), stream_handle()),
           "pdeinv_residual_kmv_mlp")
    return acc, grad


def residual_kmv(mom: torch.Tensor, wst: torch.Tensor, theta_flat: torch.Tensor, tilde_F, gamma: float):
    _require_gpu()
    n_sets = mom.shape[0]
    d = int(round(math.sqrt(theta_flat.numel() + 0.25) - 0.5))
    if tuple(mom.shape) != (n_sets, moment_len(2 * d)) or tuple(wst.shape) != (n_sets, moment_len(d)):
        raise ValueError("residual_kmv: moment shapes do not match theta's dimension")
    F = _host_f32(tilde_F)
    desc = KmvDesc(d, n_sets, float(gamma), F.ctypes.data_as(ctypes.c_void_p))
    out = torch.empty(KFP_NOUT, device=mom.device, dtype=torch.float32)
    grad = torch.empty_like(theta_flat)
    ws = torch.empty(max(1, lib().pdeinv_residual_kmv_workspace_bytes(ctypes.byref(desc)) // 8), device=mom.device,
                     dtype=torch.float64)
    mom_c, wst_c, theta_c = mom.contiguous(), wst.contiguous(), theta_flat.contiguous()
    _check(lib().pdeinv_residual_kmv(ctypes.byref(desc), _dev(mom_c, "mom", torch.float64),
                                     _dev(wst_c, "wst", torch.float64), _dev(theta_c, "theta"),
                                     _dev(ws, "ws", torch.float64), _dev(out, "out"), _dev(grad, "grad"),
                                     stream_handle()), "pdeinv_residual_kmv")
    return out, grad


def mf_desc(N: int, d: int, n_steps: int, dt: float, gamma: float, A, *, seed: int, counter_offset: int = 0,
            particle_offset: int = 0, noise_scale: float = SQRT2, random_shift: bool = True,
            noise: Optional[torch.Tensor] = None):
    p_desc, p_host = make_potential(POT_MEANFIELD_QUADRATIC, A)
    desc = SdeDesc()
    desc.n_particles = N
    desc.particle_offset = int(particle_offset)
    desc.dim = d
    desc.n_steps = int(n_steps)
    desc.dt = float(dt)
    desc.gamma = float(gamma)
    desc.noise_scale = float(noise_scale)
    desc.random_shift = int(bool(random_shift))
    desc.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    desc.counter_offset = int(counter_offset) & 0xFFFFFFFF
    desc.ld_z0 = 2 * d
    desc.potential = p_desc
    if noise is not None:
        if tuple(noise.shape) != (n_steps + 1, N, d) or not noise.is_contiguous():
            raise ValueError(f"noise must be contiguous [{n_steps + 1}, {N}, {d}]")
        desc.d_noise = _dev(noise, "noise")
    return desc, p_host


def mf_workspace(desc: SdeDesc, device) -> torch.Tensor:
    nbytes = lib().pdeinv_mf_workspace_bytes(ctypes.byref(desc))
    return torch.empty(max(nbytes // 4, 1), device=device, dtype=torch.float32)


# -----------------------------------------------------------------------------------------
# non-parametric (MLP) KFP residual
# -----------------------------------------------------------------------------------------
def residual_kfp_mlp(dims, params_flat: torch.Tensor, z_init: torch.Tensor, z_term: torch.Tensor,
                     z_0T: torch.Tensor, *, true_kind: int, true_params, gamma: float, total_time: float,
                     sigma_true: float = 1.0, world_scale: float = 1.0, chunk_rows: int = 1 << 18,
                     impl: int = MLP_IMPL_AUTO, coefficients: Optional[dict] = None, boundary_value: bool = False):
    """kinetic_fokker_planck.py:11-69 for V_hypothesis. dims = [d, W, ..., W, out] (equal hidden widths).
    Returns (acc fp64 [8], grad fp32 [P]) — sums with the reference's loss weights.
    `coefficients` overrides the per-term weights (c_nabla, c_hess, c_fric, c_true, c_init, c_term) and
    `boundary_value` makes the boundary sets weight V instead of V' (overdamped FP: residual_fp_mlp)."""
    _require_gpu()
    d, W, O = dims[0], dims[1], dims[-1]
    L = len(dims) - 2
    if L < 1 or any(w != W for w in dims[1:-1]):
        raise NotImplementedError("MLP residual: hidden layers must share one width (V_hypothesis)")
    P = lib().pdeinv_mlp_param_count(d, L, W, O)
    if params_flat.numel() != P or not params_flat.is_contiguous():
        raise ValueError(f"MLP residual: params must be a contiguous flat vector of {P} floats")
    m = 2 * d
    pi, ni, ldi = _rows(z_init, "initial", m) if z_init.shape[0] else (None, 0, m)
    pt, nt, ldt = _rows(z_term, "terminal", m) if z_term.shape[0] else (None, 0, m)
    p0, n0, ld0 = _rows(z_0T, "0T", m)
    tp = _host_f32(true_params)
    M = float(n0)
    c = dict(c_nabla=1.0 / M, c_hess=-2.0 / M, c_fric=2.0 * gamma / M, c_true=1.0 / M,
             c_init=(-2.0 / (total_time * ni)) if ni else 0.0, c_term=(2.0 / (total_time * nt)) if nt else 0.0)
    if coefficients is not None:
        c.update(coefficients)
    c = {k: v * world_scale for k, v in c.items()}
    desc = KfpMlpDesc(d, L, W, O, int(true_kind), int(tp.size // d) if true_kind == POT_GMM else 0,
                      float(sigma_true), tp.ctypes.data_as(ctypes.c_void_p), float(gamma), c["c_nabla"],
                      c["c_hess"], c["c_fric"], c["c_true"], c["c_init"], c["c_term"], int(chunk_rows),
                      int(impl), int(bool(boundary_value)))
    nbytes = lib().pdeinv_residual_kfp_mlp_workspace_bytes(ctypes.byref(desc))
    ws = torch.empty(nbytes // 4, device=z_0T.device, dtype=torch.float32)
    acc = torch.zeros(GMM_NACC, device=z_0T.device, dtype=torch.float64)
    grad = torch.zeros(P, device=z_0T.device, dtype=torch.float32)
    _check(lib().pdeinv_residual_kfp_mlp(ctypes.byref(desc), pi, ni, ldi, pt, nt, ldt, p0, n0, ld0,
                                         _dev(params_flat, "params"), _dev(ws, "ws"), _dev(acc, "acc", torch.float64),
                                         _dev(grad, "grad"), stream_handle()), "pdeinv_residual_kfp_mlp")
    return acc, grad


def fp_rows(x: torch.Tensor, unit_directions: bool) -> torch.Tensor:
    """[x_r | e_k] rows (n*d of them) or [x_r | 0] rows — pdeinv_fp_rows."""
    _require_gpu()
    d = x.shape[1]
    px, n, ldx = _rows(x, "x", d)
    out = torch.empty((n * (d if unit_directions else 1), 2 * d), device=x.device, dtype=torch.float32)
    _check(lib().pdeinv_fp_rows(px, n, ldx, d, int(bool(unit_directions)), _dev(out, "out"), stream_handle()),
           "pdeinv_fp_rows")
    return out


def residual_fp_mlp(dims, params_flat: torch.Tensor, x_init: torch.Tensor, x_term: torch.Tensor,
                    x_0T: torch.Tensor, *, tilde_F, total_time: float, world_scale: float = 1.0,
                    chunk_rows: int = 1 << 18, impl: int = MLP_IMPL_AUTO):
    """methods/consistency_instances/fokker_planck.py:33-63 for V_hypothesis:
    loss = E|grad V|^2 - 2 E[lap V] + E|grad V*|^2 + (2/T)(E_T V - E_0 V), V* = x^T F x / 2.
    The 0T rows are replicated along the d unit directions (lap V = sum_k e_k^T Hess V e_k) and go
    through the same fused residual as the kinetic case with boundary_value = 1. Returns (acc, grad)
    with the PDEINV_GMM_ACC_* slot meaning of residual_kfp_mlp (friction slot unused)."""
    d = dims[0]
    M = float(x_0T.shape[0])
    ni, nt = x_init.shape[0], x_term.shape[0]
    coef = dict(c_nabla=1.0 / (d * M), c_hess=-2.0 / M, c_fric=0.0, c_true=1.0 / (d * M),
                c_init=(-2.0 / (total_time * ni)) if ni else 0.0, c_term=(2.0 / (total_time * nt)) if nt else 0.0)
    z0 = fp_rows(x_0T, True)
    zi = fp_rows(x_init, False) if ni else torch.empty((0, 2 * d), device=x_0T.device)
    zt = fp_rows(x_term, False) if nt else torch.empty((0, 2 * d), device=x_0T.device)
    return residual_kfp_mlp(dims, params_flat, zi, zt, z0, true_kind=POT_QUADRATIC, true_params=tilde_F, gamma=0.0,
                            total_time=total_time, world_scale=world_scale, chunk_rows=chunk_rows, impl=impl,
                            coefficients=coef, boundary_value=True)


def fp_exact_sample(n: int, eig: dict, *, seed: int, t_range, counter_offset: int = 0, row_offset: int = 0,
                    device="cuda", return_t: bool = False):
    """x_r ~ N(m(t_r), P(t_r)), t_r ~ U(t_range) per sample (fokker_planck_example.py:88-96).
    eig: host arrays U [d,d], s [d], Um0 [d], B0 [d,d], B [d,d] (fp32-castable)."""
    _require_gpu()
    U, s_, Um0, B0, B = (_host_f32(eig[k]) for k in ("U", "s", "Um0", "B0", "B"))
    d = s_.size
    out = torch.empty((int(n), d), device=device, dtype=torch.float32)
    t_out = torch.empty(int(n), device=device, dtype=torch.float32) if return_t else None
    lo, hi = (float(t_range), float(t_range)) if np.ndim(t_range) == 0 else (float(t_range[0]), float(t_range[1]))
    _check(lib().pdeinv_fp_exact_sample(int(n), d, int(seed) & 0xFFFFFFFFFFFFFFFF, int(counter_offset) & 0xFFFFFFFF,
                                        int(row_offset), lo, hi, *(a.ctypes.data_as(ctypes.c_void_p)
                                                                   for a in (U, s_, Um0, B0, B)),
                                        _dev(out, "out"), _dev(t_out, "t_out"), stream_handle()),
           "pdeinv_fp_exact_sample")
    return (out, t_out) if return_t else out


def adam_update(params: torch.Tensor, grad: torch.Tensor, mu: torch.Tensor, nu: torch.Tensor, *, lr: float,
                b1: float, b2: float, eps: float, weight_decay: float, count: int) -> None:
    """In-place fused add_decayed_weights + adam + apply_updates on contiguous fp32 device tensors."""
    _require_gpu()
    n = params.numel()
    for t, name in ((params, "params"), (grad, "grad"), (mu, "mu"), (nu, "nu")):
        if t.numel() != n or not t.is_contiguous():
            raise ValueError(f"adam_update: {name} must be contiguous with {n} elements")
    _check(lib().pdeinv_adam_update(_dev(params, "params"), _dev(grad, "grad"), _dev(mu, "mu"), _dev(nu, "nu"), n,
                                    float(lr), float(b1), float(b2), float(eps), float(weight_decay), int(count),
                                    stream_handle()), "pdeinv_adam_update")


def realnvp_desc(dim: int, masks, embed_time_dim: int, ignore_time: bool, soft_init: float, activation: str,
                 base_mean, base_inv_cov, base_log_det: float):
    """(descriptor, keep-alive host arrays) for pdeinv_realnvp_* ."""
    if activation not in ACTIVATIONS:
        raise NotImplementedError(f"RealNVP activation '{activation}' (prelu has parameters; not supported)")
    m = _host_f32(masks)
    mu = _host_f32(base_mean)
    ic = _host_f32(base_inv_cov)
    desc = RealNvpDesc(int(dim), int(m.size // dim), int(embed_time_dim), int(bool(ignore_time)), float(soft_init),
                       ACTIVATIONS[activation], m.ctypes.data_as(ctypes.c_void_p), mu.ctypes.data_as(ctypes.c_void_p),
                       ic.ctypes.data_as(ctypes.c_void_p), float(base_log_det))
    return desc, (m, mu, ic)


def realnvp_param_count(desc) -> int:
    n = lib().pdeinv_realnvp_param_count(ctypes.byref(desc))
    if n < 0:
        raise ValueError("RealNVP: bad descriptor")
    return int(n)


def realnvp_logdensity(desc, params: torch.Tensor, t: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """log p_t(x) for rows x [n, dim] and times t [n] (or a 0-d / [1] t broadcast)."""
    _require_gpu()
    n = x.shape[0]
    if params.numel() != realnvp_param_count(desc) or not params.is_contiguous():
        raise ValueError("RealNVP: params must be a contiguous flat vector of pdeinv_realnvp_param_count floats")
    t = t.reshape(-1)
    if t.numel() not in (1, n):
        raise ValueError("RealNVP: t must have one entry per row or a single entry")
    px, _, ld = _rows(x, "x", desc.dim)
    out = torch.empty(n, device=x.device, dtype=torch.float32)
    t = t.contiguous()
    _check(lib().pdeinv_realnvp_logdensity(ctypes.byref(desc), _dev(params, "params"), _dev(t, "t"),
                                           0 if t.numel() == 1 else 1, px, n, ld, _dev(out, "out"),
                                           stream_handle()), "pdeinv_realnvp_logdensity")
    return out


def realnvp_value_and_grad(desc, params: torch.Tensor, t: torch.Tensor, x: torch.Tensor):
    """(loss, grad): loss = -mean log p_t(x) (log_density_estimation.py:51-58), grad flat like params."""
    _require_gpu()
    n = x.shape[0]
    P = realnvp_param_count(desc)
    if params.numel() != P or not params.is_contiguous():
        raise ValueError("RealNVP: params must be a contiguous flat vector of pdeinv_realnvp_param_count floats")
    if n < 1:
        raise ValueError("RealNVP: value_and_grad needs at least one sample")
    t = t.reshape(-1)
    if t.numel() not in (1, n):
        raise ValueError("RealNVP: t must have one entry per row or a single entry")
    px, _, ld = _rows(x, "x", desc.dim)
    ws_bytes = int(lib().pdeinv_realnvp_grad_workspace(ctypes.byref(desc), n))
    ws = torch.empty((ws_bytes + 3) // 4, device=x.device, dtype=torch.float32)
    loss = torch.empty((), device=x.device, dtype=torch.float32)
    grad = torch.empty(P, device=x.device, dtype=torch.float32)
    t = t.contiguous()
    _check(lib().pdeinv_realnvp_value_and_grad(ctypes.byref(desc), _dev(params, "params"), _dev(t, "t"),
                                               0 if t.numel() == 1 else 1, px, n, ld, _dev(loss, "loss"),
                                               _dev(grad, "grad"), _dev(ws, "workspace"), ws_bytes,
                                               stream_handle()), "pdeinv_realnvp_value_and_grad")
    return loss, grad


KMV_PATHS = {0: "pair_tiles_mfma", 1: "pair_ring", 2: "fused_rows_mfma", 3: "library_rocblas"}


def kmv_mlp_path(dims, impl: int = MLP_IMPL_AUTO) -> str:
    """Which kernels pdeinv_residual_kmv_mlp runs for this Phi net and impl (pdeinv_kmv_mlp_path): the 16-pair
    MFMA tiles, the register-ring pair kernels, pair rows through the fused MFMA residual, or rocBLAS."""
    d, W, O, L = dims[0], dims[1], dims[-1], len(dims) - 2
    F = np.zeros((d, d), dtype=np.float32)
    desc = KmvMlpDesc(d, L, W, O, 1, 1, 1.0, F.ctypes.data_as(ctypes.c_void_p), 0, int(impl))
    p = int(lib().pdeinv_kmv_mlp_path(ctypes.byref(desc)))
    if p < 0:
        raise NotImplementedError(f"kmv_mlp: unsupported shape {dims} / impl {impl}")
    return KMV_PATHS[p]


def rocblas_calls() -> int:
    """Residual calls served by rocBLAS in this process (pdeinv_rocblas_calls): only impl = LIBRARY adds to it."""
    return int(lib().pdeinv_rocblas_calls())


def mlp_fused_supported(dims) -> bool:
    """True when residual_kfp_mlp (impl = AUTO) runs the hand-written fused MFMA path for this V_hypothesis shape —
    compiled shapes and the zero-padded envelope (pdeinv_mlp_fused_supported). Not a statement about the KMV pair
    tiles (kmv_pair_tiles_supported)."""
    return bool(lib().pdeinv_mlp_fused_supported(dims[0], len(dims) - 2, dims[1], dims[-1]))


def kfp_terms_finalize(acc: torch.Tensor, grad: torch.Tensor, gamma: float) -> torch.Tensor:
    out = torch.empty(KFP_NOUT, device=acc.device, dtype=torch.float32)
    _check(lib().pdeinv_kfp_terms_finalize(_dev(acc, "acc", torch.float64), _dev(grad, "grad"), grad.numel(),
                                           float(gamma), _dev(out, "out"), stream_handle()), "pdeinv_kfp_terms_finalize")
    return out


def gather_random_step(traj_tm: torch.Tensor, *, seed: int, ctr: int = 0, return_t: bool = False):
    """One uniformly drawn step per particle from a time-major trajectory [n, N, m] -> [N, m]."""
    _require_gpu()
    n, N, m = traj_tm.shape
    if not traj_tm.is_contiguous():
        raise ValueError("trajectory must be contiguous time-major [n, N, m]")
    out = torch.empty((N, m), device=traj_tm.device, dtype=torch.float32)
    t = torch.empty(N, device=traj_tm.device, dtype=torch.int32) if return_t else None
    _check(lib().pdeinv_gather_random_step(_dev(traj_tm, "traj"), N, n, m, int(seed) & 0xFFFFFFFFFFFFFFFF,
                                           int(ctr) & 0xFFFFFFFF, _dev(out, "out"), _dev(t, "t", torch.int32),
                                           stream_handle()), "pdeinv_gather_random_step")
    return (out, t) if return_t else out
