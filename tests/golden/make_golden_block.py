"""Golden vectors for the block-diagonal variational family (`ziggy/hipgp.py:527-691`,
SURVEY §8(f) row 3), made by running the *reference* `BlockToeplitzGP` in this container
through the same in-memory torch-1.4 shim as `make_golden.py` (no reference file modified,
no reference source copied; the fixtures are data only).

G11: 2-D 11x9 grid (expanded 20x16), Matern-3/2 (1, .2), blocks 4x4 (16 points), 48 obs,
     shared noise (log_noise2), theta2 = -1/2 S0^{-1} with random SPD blocks S0.
G12: 3-D 6x5x4 grid (expanded 10x8x6), SqExp (1, .3), blocks 2x2x3 (12 points), 40 obs,
     per-observation noise (noise_std_batch).

Recorded: grams, kn, theta1/theta2, the block index table, elbo, theta grads, knSkn,
predict mu/sig.

Usage:  python tests/golden/make_golden_block.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, _np, import_reference  # noqa: E402


def _spd_blocks(rs, nblk, bs, dtype):
    A = rs.randn(nblk, bs, bs) / np.sqrt(bs)
    S0 = 0.05 * np.einsum("bij,bkj->bik", A, A) + 0.02 * np.eye(bs)[None]
    return torch.tensor(-0.5 * np.linalg.inv(S0), dtype=dtype)


def gen_case(zk, hg, dtype, tag, name, dims, kern, params, blocks, nobs, per_obs_noise, seed):
    torch.manual_seed(seed)
    rs = np.random.RandomState(seed)
    xgrids = [torch.linspace(-1, 1, m, dtype=dtype) for m in dims]
    mod = hg.BlockToeplitzGP(kern, xgrids, num_obs=10 * nobs, block_sizes=list(blocks),
                             sig2_init=params[0], ell_init=params[1], noise2_init=.05,
                             learn_kernel=False, dtype=dtype)
    with torch.no_grad():
        mod.global_theta1.copy_(torch.tensor(rs.randn(mod.Mprime, 1) * .3, dtype=dtype))
        mod.global_theta2.copy_(_spd_blocks(rs, mod.num_blocks, mod.block_size, dtype))
    xobs = torch.tensor(rs.rand(nobs, len(dims)) * 1.8 - .9, dtype=dtype)
    yobs = torch.tensor(rs.randn(nobs, 1), dtype=dtype)
    nstd = torch.tensor(.1 + .2 * rs.rand(nobs, 1), dtype=dtype) if per_obs_noise else None
    Knm, Knn = mod._make_grams(xobs)
    kn = mod.compute_kn(Knm, maxiter_cg=20)
    qm, qS = mod.standard_variational_params()
    out = {f"grid{i}": _np(g) for i, g in enumerate(xgrids)}
    out.update({"dims": np.array(dims), "blocks": np.array(blocks), "params": np.array(params),
                "num_obs": np.array(10 * nobs), "noise2": np.array(.05),
                "xobs": _np(xobs), "yobs": _np(yobs), "Knm": _np(Knm), "Knn_diag": _np(Knn),
                "kn": _np(kn), "theta1": _np(mod.global_theta1), "theta2": _np(mod.global_theta2),
                "block_idx": _np(mod.block_idx), "qm": _np(qm), "qS": _np(qS),
                "knSkn": _np(mod.compute_knSkn(kn, qS)),
                "kl": np.array(float(mod.get_kl_to_prior(qm, qS)))})
    if nstd is not None:
        out["noise_std"] = _np(nstd)
    an = mod.compute_batch_an(xobs, yobs, nstd, qm=qm, qS=qS, Knm=Knm, Knn_diag=Knn, kn=kn)
    out["batch_an"] = _np(an)
    elbo = mod.elbo_and_grad(xobs, yobs, noise_std_batch=nstd, maxiter_cg=20)
    out["elbo"] = np.array(float(elbo))
    out["theta1_grad"] = _np(mod.global_theta1.grad)
    out["theta2_grad"] = _np(mod.global_theta2.grad)
    mu, sig = mod.predict(xobs[:20], maxiter_cg=50)
    out["pred_mu"] = _np(mu)
    out["pred_sig"] = _np(sig)
    np.savez_compressed(os.path.join(OUT, f"{name}_{tag}.npz"), **out)


def main():
    zk, tt, te, cg, hg = import_reference()
    torch.set_num_threads(8)
    for dtype, tag in ((torch.float64, "f64"), (torch.float32, "f32")):
        gen_case(zk, hg, dtype, tag, "G11", (11, 9), zk.Matern(nu=1.5, dtype=dtype), (1., .2),
                 (4, 4), 48, False, 11)
        gen_case(zk, hg, dtype, tag, "G12", (6, 5, 4), zk.SqExp(dtype=dtype), (1., .3),
                 (2, 2, 3), 40, True, 12)
        print("wrote", tag)


if __name__ == "__main__":
    main()
