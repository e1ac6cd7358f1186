"""Block-diagonal variational family (`ziggy/hipgp.py:527-691`): the NumPy
oracle against the reference's own outputs (G11 2-D shared noise, G12 3-D per-observation
noise; tests/golden/make_golden_block.py ran the reference BlockToeplitzGP)."""
import numpy as np
import pytest

from golden_cases import load, rel_err
from oracle import ziggy_oracle as zo


def _noise(fx):
    if "noise_std" in fx:
        s = fx["noise_std"].reshape(-1)
        return 1 / s ** 2, np.log(s)
    return 1 / fx["noise2"], 0.5 * np.log(fx["noise2"])


@pytest.mark.parametrize("name", ["G11", "G12"])
def test_block_index_matches_reference(name):
    fx = load(name, "f64")
    exp = [2 * int(m) - 2 for m in fx["dims"]]
    idx = zo.block_index(exp, fx["blocks"])
    assert np.array_equal(idx, fx["block_idx"])


@pytest.mark.parametrize("name", ["G11", "G12"])
def test_block_kn_and_natgrad(name):
    fx = load(name, "f64")
    grids = [fx[f"grid{i}"] for i in range(len(fx["dims"]))]
    kind, nu = ("matern", 1.5) if name == "G11" else ("sqexp", None)
    kf = lambda x, y: zo.kernel_eval(kind, x, y, tuple(fx["params"]), nu=nu)
    T = zo.ToeplitzOracle(zo.toeplitz_column(grids, kf, 1e-3), tuple(int(m) for m in fx["dims"]))
    kn = zo.compute_kn(T, fx["Knm"], maxiter_cg=20, tol=1e-8)
    assert rel_err(kn, fx["kn"]) < 1e-8
    iv, lsd = _noise(fx)
    idx = fx["block_idx"]
    elbo, g1, g2, an, knSkn = zo.block_elbo_and_grad(fx["kn"], fx["yobs"], fx["Knn_diag"], fx["theta1"],
                                                     fx["theta2"], idx, float(fx["num_obs"]), iv, lsd)
    assert rel_err(knSkn, fx["knSkn"]) < 1e-10
    if fx["batch_an"].ndim == 2:
        # reference quirk (hipgp.py:396-408): with per-observation noise, log(noise_std) keeps
        # its (bsz, 1) shape and batch_an broadcasts to (bsz, bsz) [i, j] = a_j + lsd_j - lsd_i;
        # its mean (the ELBO term) equals the mean of the per-observation a_n.
        an = (an + lsd)[None, :] - lsd[:, None]
    assert rel_err(an, fx["batch_an"]) < 1e-10
    assert abs(elbo - float(fx["elbo"])) < 1e-10 * abs(float(fx["elbo"]))
    assert rel_err(g1, fx["theta1_grad"]) < 1e-10
    assert rel_err(g2, fx["theta2_grad"]) < 1e-10
    qm = zo.block_diag_multiply(np.linalg.inv(-2 * fx["theta2"]), fx["theta1"].T, idx).T
    assert rel_err(qm, fx["qm"]) < 1e-10
    assert abs(zo.block_kl_to_standard(qm, fx["qS"]) - float(fx["kl"])) < 1e-9 * abs(float(fx["kl"]))
