"""Plugin registry (registry.py of the reference): problem and method lookup by config name."""
from example_problems.fokker_planck_example import FokkerPlanck
from example_problems.kinetic_fokker_planck_example_GMM import KineticFokkerPlanck as KFPGMM
from example_problems.kinetic_fokker_planck_example_OU import KineticFokkerPlanck as KFPOU
from example_problems.kinetic_mckean_vlasov_example_quadratic import KineticMcKeanVlasov as KMVOU
from methods.consistency import ConsistencyBased

KineticFokkerPlanckPotential = {
    "Quadratic": KFPOU,
    "GMM": KFPGMM,
}

KineticMcKeanVlasovPotential = {
    "Quadratic": KMVOU,
}


def get_pde_instance(cfg):
    """registry.py:18-26. The reference *returns* NotImplementedError for an unknown name
    (registry.py:25-26); here it is raised, so the failure is not deferred."""
    name = cfg.pde_instance.name
    if name == "Fokker-Planck":
        return FokkerPlanck
    if name == "Kinetic-Fokker-Planck":
        return KineticFokkerPlanckPotential[cfg.pde_instance.potential]
    if name == "Kinetic-McKean-Vlasov":
        return KineticMcKeanVlasovPotential[cfg.pde_instance.potential]
    raise NotImplementedError(f"pde_instance '{name}' is not part of this build")


def get_method(cfg):
    if cfg.solver.name == "ConsistencyBased":
        return ConsistencyBased
    raise NotImplementedError
