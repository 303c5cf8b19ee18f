"""Data-parallel plumbing: one process per GPU, torch.distributed over RCCL (backend "nccl").

Replaces the reference's `jax.pmap(value_and_grad_fn, in_axes=(None, 0))` followed by
`jnp.mean(axis=0)` over the device axis (core/trainer.py:44-53). Particles are sharded by
contiguous global-id ranges, so every rank's Philox streams are those of a single-process run
over the same ids. The only exchanges are one all-reduce per residual evaluation (the fp64
moment / loss-term sums and the parameter gradient, a few hundred bytes) and, for
McKean–Vlasov, one all-reduce per simulate of [count, sum z0, sum of every update's noise]
(utils/mean_field.py; the per-update driver instead all-reduces sum(x) once per update).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def _forced() -> bool:
    """PDEINV_DIST_FORCE=1: take the distributed path (process group + every all-reduce call site) even
    at world size 1 — lets a one-GPU box execute the RCCL data path (tests/test_gpu_multirank.py)."""
    return os.environ.get("PDEINV_DIST_FORCE", "0") == "1"


def is_distributed() -> bool:
    return dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or _forced())


def rank() -> int:
    return dist.get_rank() if is_distributed() else 0


def world_size() -> int:
    return dist.get_world_size() if is_distributed() else 1


def init_from_env(backend: str = None) -> bool:
    """Initialise from torchrun's env (RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT); no-op for one rank."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if (ws <= 1 and not _forced()) or dist.is_initialized():
        return dist.is_initialized()
    if ws <= 1 and not all(k in os.environ for k in ("MASTER_ADDR", "MASTER_PORT")):
        raise RuntimeError("PDEINV_DIST_FORCE=1 forces the distributed path at world size 1, which needs the "
                           "torch.distributed.run rendezvous (MASTER_ADDR / MASTER_PORT); launch under "
                           "torch.distributed.run or unset PDEINV_DIST_FORCE")
    backend = os.environ.get("PDEINV_DIST_BACKEND", backend)  # test override (e.g. gloo on one GPU)
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if torch.cuda.is_available():
        torch.cuda.set_device(local_device())
    dist.init_process_group(backend=backend)
    return True


def local_device() -> int:
    """LOCAL_RANK modulo the visible devices (lets a test run several ranks on one GPU)."""
    n = max(torch.cuda.device_count(), 1)
    return int(os.environ.get("LOCAL_RANK", "0")) % n


def shard(n_global: int, r: int = None, w: int = None):
    """Contiguous [offset, offset + n) share of n_global units for rank r of w."""
    r = rank() if r is None else r
    w = world_size() if w is None else w
    base, rem = divmod(int(n_global), w)
    n = base + (1 if r < rem else 0)
    off = r * base + min(r, rem)
    return off, n


def allreduce_sum(t: torch.Tensor) -> torch.Tensor:
    if is_distributed():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def allreduce_mean(t: torch.Tensor) -> torch.Tensor:
    if is_distributed():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t /= dist.get_world_size()
    return t


def allreduce_max_scalar(x: float, device=None) -> float:
    if not is_distributed():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier():
    if is_distributed():
        dist.barrier()
