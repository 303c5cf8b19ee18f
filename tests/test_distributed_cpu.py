"""World-size-2 gloo tests of the data-parallel plumbing (CPU): the all-reduce helpers, rank
sharding, and that sharded fp64 moment sums reduce to the single-process moments (the
reduction behind every multi-GPU residual)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "pde-inverse-problem_amd"), root]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from utils import distributed as pd
    from oracle import numpy_ref as nr
    pd.init_from_env("gloo")
    try:
        assert pd.is_distributed() and pd.rank() == rank and pd.world_size() == world
        data = np.random.default_rng(0).standard_normal((1001, 6))
        off, n = pd.shard(len(data))
        local = torch.as_tensor(nr.moments(data[off:off + n]))
        total = pd.allreduce_sum(local.clone())
        ok_sum = np.allclose(total.numpy(), nr.moments(data), rtol=1e-12)
        mean = pd.allreduce_mean(torch.tensor([float(rank)], dtype=torch.float64))
        mx = pd.allreduce_max_scalar(float(rank) * 3.0)
        pd.barrier()
        q.put((rank, ok_sum, float(mean.item()), mx))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2_reductions():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(100)
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert [r[1] for r in res] == [True, True]
    assert all(abs(r[2] - 0.5) < 1e-12 for r in res) and all(r[3] == 3.0 for r in res)


def _ramp_worker(rank, world, port, q):
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "pde-inverse-problem_amd"), root]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from utils import distributed as pd
    import bench
    pd.init_from_env("gloo")
    try:
        calls = [0]

        def ramp():  # a step with a collective inside, slower on rank 1: its own clock would stop it earlier
            time.sleep(0.004 * (1 + 3 * rank))
            pd.allreduce_sum(torch.ones(3, dtype=torch.float64))
            calls[0] += 1

        rounds = bench.run_ramp(ramp, None, seconds=0.25, sync=lambda: None)
        pd.allreduce_sum(torch.ones(1, dtype=torch.float64))  # the warmup / timed steps that follow still pair up
        pd.barrier()
        q.put((rank, rounds, calls[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_bench_ramp_rounds_agree_across_ranks():
    """bench.run_ramp: ranks whose ramp steps take different times (and hold a collective) run the same number
    of rounds, so the collectives of the ramp, the warmup and the timed region pair up (no hang)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ramp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(100)
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert res[0][1] == res[1][1] >= 1 and res[0][2] == res[1][2] == 8 * res[0][1]
