"""MFMA pair-tile kernels vs the register-ring kernels on the same inputs (acc slots, gradient)."""
import os
import sys
import json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pde-inverse-problem_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from utils import native  # noqa: E402


def run(d, n, n_t, W, L, O=0):
    from core.model import V_hypothesis
    from utils import prng
    from example_problems.kinetic_mckean_vlasov_example_quadratic import dlogrho_coefficients
    from example_problems.kinetic_fokker_planck_example_OU import initialize_configuration
    net = V_hypothesis(output_dim=1, hidden_dims=[W] * L)
    params = net.init(prng.PRNGKey(11), np.zeros(d), device="cuda")
    flat, dims = net.flat(params), net.dims(d)
    if O:  # a custom output width: random parameters of that shape
        dims = dims[:-1] + [O]
        npar = sum(dims[i] * dims[i + 1] + dims[i + 1] for i in range(len(dims) - 1))
        flat = torch.as_tensor(0.4 * np.random.default_rng(3).standard_normal(npar), dtype=torch.float32, device="cuda")
    ic = initialize_configuration(d)
    z = torch.as_tensor(np.random.default_rng(0).standard_normal((n * n_t, 2 * d)), dtype=torch.float32, device="cuda")
    tau = np.linspace(0.3, 1.7, n_t)
    coef = torch.as_tensor(dlogrho_coefficients(tau, ic, d), dtype=torch.float32, device="cuda")
    _, ds = native.kmv_weights(d, 1.0, coef, z, n_t, n, 2 * d, n_t * 2 * d, want_ds=True)
    out = {}
    for impl in ("mfma", "ring"):
        acc, g = native.residual_kmv_mlp(dims, flat, z, n_t, n, 2 * d, n_t * 2 * d, ds, ic["tilde_F"], 1.0,
                                         impl=native.MLP_IMPL_FUSED if impl == "mfma" else native.MLP_IMPL_PAIRS_RING)
        torch.cuda.synchronize()
        out[impl] = (acc.double().cpu().numpy(), g.double().cpu().numpy())
    a0, g0 = out["mfma"]
    a1, g1 = out["ring"]
    print(json.dumps({"d": d, "n": n, "n_t": n_t, "W": W, "L": L, "O": dims[-1],
                      "acc_mfma": [round(float(v), 6) for v in a0[:8]], "acc_ring": [round(float(v), 6) for v in a1[:8]],
                      "grad_rel": float(np.abs(g0 - g1).max() / (np.abs(g1).max() + 1e-30))}), flush=True)


if __name__ == "__main__":
    native.lib()
    for c in sys.argv[1:]:
        run(*[int(v) for v in c.split(",")])
