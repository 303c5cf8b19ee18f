"""Time the general-Phi KMV residual (pdeinv_residual_kmv_mlp) on the reference's runnable KMV recipe
(scripts/parametric/KMV/run_quadratic_online.sh: d = 2, one time stamp, 5 000 particles -> 25 M pairs)
with the reference's default hypothesis net (configurations/neural_network/MLP.yaml: width 20, 8 layers)
and on a wider net; and the KFP MLP residual at the default shape. Prints one JSON line per case."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pde-inverse-problem_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from utils import native  # noqa: E402


def run(d, n, n_t, W, L, reps=3, impl=0):
    from core.model import V_hypothesis
    from utils import prng
    from example_problems.kinetic_mckean_vlasov_example_quadratic import dlogrho_coefficients
    from example_problems.kinetic_fokker_planck_example_OU import initialize_configuration
    net = V_hypothesis(output_dim=1, hidden_dims=[W] * L)
    params = net.init(prng.PRNGKey(11), np.zeros(d), device="cuda")
    flat, dims = net.flat(params), net.dims(d)
    ic = initialize_configuration(d)
    z = torch.as_tensor(np.random.default_rng(0).standard_normal((n * n_t, 2 * d)), dtype=torch.float32, device="cuda")
    tau = np.linspace(0.3, 1.7, n_t)
    coef = torch.as_tensor(dlogrho_coefficients(tau, ic, d), dtype=torch.float32, device="cuda")
    _, ds = native.kmv_weights(d, 1.0, coef, z, n_t, n, 2 * d, n_t * 2 * d, want_ds=True)
    f = lambda: native.residual_kmv_mlp(dims, flat, z, n_t, n, 2 * d, n_t * 2 * d, ds, ic["tilde_F"], 1.0, impl=impl)
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        acc, g = f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    pairs = n * n * n_t
    print(json.dumps({"case": "kmv_mlp", "impl": impl, "d": d, "n": n, "n_time": n_t, "dims": dims, "pairs": pairs, "ms": ms,
                      "pairs_per_s": pairs / (ms / 1e3), "path": native.kmv_mlp_path(dims, impl),
                      "loss_acc0": float(acc[0]), "grad_norm": float(g.norm())}), flush=True)


if __name__ == "__main__":
    native.lib()
    cases = [(2, 5000, 1, 20, 8, 2), (2, 5000, 1, 20, 8, 1), (2, 2000, 3, 20, 8, 2)]
    if len(sys.argv) > 1:
        cases = [tuple(int(v) for v in c.split(",")) for c in sys.argv[1:]]
    for c in cases:
        run(*c[:5], impl=c[5])
