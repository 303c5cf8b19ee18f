"""Entry point (main.py of the reference): compose the config, build problem / method / model /
optimizer, train. Same CLI override grammar as the reference's Hydra entry (main.py:32):

    python main.py pde_instance=kinetic_fokker_planck pde_instance.potential=GMM \
        pde_instance.sample_mode=offline train.optimizer.learning_rate.initial=1e-2

Multi-GPU: torchrun --nproc-per-node N main.py ... (one process per GPU, RCCL), the counterpart
of backend.use_pmap_train=True.
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from core.trainer import JaxTrainer, get_optimizer  # noqa: E402
from registry import get_method, get_pde_instance  # noqa: E402
from utils import config as config_lib  # noqa: E402
from utils import distributed as dist  # noqa: E402
from utils import prng  # noqa: E402


def run(cfg, log_path=None, number_of_iterations=None):
    seeds_keys = ["rng_problem", "rng_method", "rng_trainer", "rng_log_density"]
    seeds = dict(zip(seeds_keys, prng.split(prng.PRNGKey(cfg.seed), len(seeds_keys))))  # main.py:43-44
    pde_instance = get_pde_instance(cfg)(cfg=cfg, rng=seeds["rng_problem"])
    method = get_method(cfg)(pde_instance=pde_instance, cfg=cfg, rng=seeds["rng_method"])
    net, params = method.create_model_fn()
    optimizer = get_optimizer(cfg.train.optimizer)
    trainer = JaxTrainer(cfg=cfg, method=method, rng=seeds["rng_trainer"], forward_fn=net.apply, params=params,
                         optimizer=optimizer, log_path=log_path)
    params = trainer.fit(number_of_iterations)
    return trainer, params


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    cfg = config_lib.compose("config", argv)
    dist.init_from_env()
    import torch
    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    name = f"{cfg.pde_instance.domain_dim}D-{cfg.pde_instance.name}-{cfg.pde_instance.potential}"
    log_path = os.environ.get("PDEINV_LOG", f"{name}-{cfg.solver.name}.jsonl")
    trainer, _ = run(cfg, log_path=log_path)
    if dist.rank() == 0 and trainer.history:
        print({k: v for k, v in trainer.history[-1].items()})


if __name__ == "__main__":
    main()
