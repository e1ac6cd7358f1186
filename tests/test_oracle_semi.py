"""CPU oracle vs the reference's line-integral cross covariance:
golden vectors from tests/golden/make_golden_semi.py (the reference run in this container)."""
import numpy as np
import pytest

from golden_cases import SEMI_CASES, SEMI_KERNELS, load, grids_of, rel_err
from oracle import ziggy_oracle as zo


@pytest.mark.parametrize("name", sorted(SEMI_CASES))
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_semi_mc_and_analytic(name, tag):
    fx = load(name, tag)
    params = SEMI_CASES[name]
    xin = zo.grid_points(grids_of(fx)).astype(fx["x"].dtype)
    tol = 1e-12 if tag == "f64" else 3e-6
    for key, (kind, nu) in SEMI_KERNELS.items():
        for npts in (1, 10):
            u = float(fx[f"u_{key}_n{npts}"][0])
            got = zo.k_semi_mc(kind, xin, fx["x"], params, npts, u, nu=nu)
            assert got.shape == fx[f"mc_{key}_n{npts}"].shape
            assert rel_err(got, fx[f"mc_{key}_n{npts}"]) < tol, (key, npts)
    got = zo.k_semi_sqexp(xin, fx["x"], params)
    # the analytic form subtracts two normal CDFs: in fp32 the cancellation error scales with
    # coef (<= max Knm), so compare relative to the largest entry
    assert rel_err(got, fx["semi_sqexp"]) < (1e-12 if tag == "f64" else 2e-5)


@pytest.mark.parametrize("name", sorted(SEMI_CASES))
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_doubly_diag_interp(name, tag):
    fx = load(name, tag)
    params = SEMI_CASES[name]
    for key in SEMI_KERNELS:
        table = (fx[f"dd_grid_{key}"], fx[f"dd_knn_{key}"], fx[f"dd_slopes_{key}"])
        got = zo.doubly_diag(fx["x"], params, table)
        assert rel_err(got, fx[f"dd_{key}"]) < (1e-12 if tag == "f64" else 2e-6), key


@pytest.mark.parametrize("key", ["sqexp", "matern1.5"])
def test_doubly_diag_table(key):
    """The oracle's dblquad table equals the reference's (both stored as float32)."""
    fx = load("G9", "f64")
    kind, nu = SEMI_KERNELS[key]
    grid, knn, slopes = zo.doubly_diag_table(kind, nu=nu)
    np.testing.assert_array_equal(grid, fx[f"dd_grid_{key}"].astype(np.float32))
    assert rel_err(knn, fx[f"dd_knn_{key}"]) < 1e-6
    assert rel_err(slopes, fx[f"dd_slopes_{key}"]) < 1e-6


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_model_integrated_G10(tag):
    """Knm (analytic), Knn_diag and kn = R^T K^-1 Knm^T of the reference's 3-D
    MeanFieldToeplitzGP with line-integral observations."""
    fx = load("G10", tag)
    grids = grids_of(fx)
    dims = tuple(len(g) for g in grids)
    xin = zo.grid_points(grids).astype(fx["x"].dtype)
    params = (1., .1)
    Knm = zo.k_semi_sqexp(xin, fx["x"], params)
    assert rel_err(Knm, fx["Knm"]) < (1e-12 if tag == "f64" else 2e-5)
    t = load("G8", tag)
    table = (t["dd_grid_sqexp"], t["dd_knn_sqexp"], t["dd_slopes_sqexp"])
    assert rel_err(zo.doubly_diag(fx["x"], params, table), fx["Knn_diag"]) < (1e-12 if tag == "f64" else 2e-6)
    if tag == "f64":
        kf = lambda x, y: zo.kernel_eval("sqexp", x, y, params)
        T = zo.ToeplitzOracle(zo.toeplitz_column(grids, kf, 1e-3), dims)
        kn = zo.compute_kn(T, fx["Knm"], maxiter_cg=20, tol=1e-8)
        assert rel_err(kn, fx["kn"]) < 1e-8
