"""CPU oracle vs the reference's own outputs (golden vectors made by running /root/reference).

These pin the oracle before it is trusted as the checker for the HIP path."""
import numpy as np
import pytest

from golden_cases import GRID_CASES, CLAMPED, load, grids_of, rel_err, op_ok, chaotic_bound
from oracle import ziggy_oracle as zo


def _kfun(kind, nu, params):
    return lambda x, y: zo.kernel_eval(kind, x, y, params, nu=nu)


@pytest.mark.parametrize("name", sorted(GRID_CASES))
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_grid_case_ops(name, tag):
    kind, nu, params, jit = GRID_CASES[name]
    fx = load(name, tag)
    grids = grids_of(fx)
    dims = tuple(len(g) for g in grids)
    col = zo.toeplitz_column(grids, _kfun(kind, nu, params), jit).astype(fx["column"].dtype)
    tol = 1e-12 if tag == "f64" else 2e-6
    assert rel_err(col, fx["column"]) < tol
    T = zo.ToeplitzOracle(fx["column"], dims)
    assert T.C.shape == fx["C"].shape
    np.testing.assert_array_equal(T.C, fx["C"])
    assert T.Mp == int(np.prod(zo.expanded_dims(dims)))
    # D carries the FFT's rounding noise (~eps * max D): compare D-derived quantities in
    # D-space, relative to max D (1/D amplifies the noise where D is near the clamp).
    dtol = 1e-12 if tag == "f64" else 1e-6
    assert rel_err(T.D, fx["D"]) < dtol
    assert rel_err(T.D_sqrt ** 2, fx["D_sqrt"].astype(np.float64) ** 2) < dtol
    assert rel_err(1 / T.Di.astype(np.float64), 1 / fx["Di"].astype(np.float64)) < dtol
    if tag == "f64":      # same clamp set (in fp32 the set is rounding-noise dependent)
        assert np.array_equal(T.D <= 1e-6, fx["D"] <= 1e-6)
    for key, fn, x in (("Kv", T.matmul_K, fx["v"]), ("Cinv_v", T.matmul_Cinv, fx["v"]),
                       ("RTv", T.matmul_RT, fx["v"]), ("Rw", T.matmul_R, fx["w"])):
        y = fn(x)
        assert y.shape == fx[key].shape
        if tag == "f64":
            assert rel_err(y, fx[key]) < 1e-9, key
        elif not (name in CLAMPED and key in ("Cinv_v", "Rw")):
            # (clamped fp32: 1/D at noise-level eigenvalues is rounding-chaotic, see CLAMPED)
            assert op_ok(y, fx[key], load(name, "f64")[key]), key


@pytest.mark.parametrize("name", sorted(GRID_CASES))
def test_grid_case_solves(name):
    f64 = load(name, "f64")
    f32 = load(name, "f32")
    dims = tuple(len(g) for g in grids_of(f64))
    T64 = zo.ToeplitzOracle(f64["column"], dims)
    T32 = zo.ToeplitzOracle(f32["column"], dims)
    for mi in (1, 2, 5, 20):
        key = f"solve_p1_it{mi}"
        x64 = T64.solve(f64["v"], do_precond=True, maxiter=mi, tol=1e-8)
        chaotic = name in CLAMPED and mi == 20
        if chaotic:
            # the reference's own chaotic spread sets the bound (golden_cases.chaotic_bound)
            assert rel_err(x64, f64[key]) <= chaotic_bound(name, "f64", key), (key, rel_err(x64, f64[key]))
        else:
            assert rel_err(x64, f64[key]) < 1e-8, key
        if name not in CLAMPED:
            x32 = T32.solve(f32["v"], do_precond=True, maxiter=mi, tol=1e-8)
            # oracle fp32 error no worse than 4x the reference's own fp32 error (+ floor)
            e_me = np.linalg.norm(x32.astype(np.float64) - f64[key])
            e_ref = np.linalg.norm(f32[key].astype(np.float64) - f64[key])
            assert e_me <= 4 * e_ref + 1e-6 * np.linalg.norm(f64[key]), (key, e_me, e_ref)
    x = T64.solve(f64["v"], do_precond=False, maxiter=5, tol=1e-8)
    assert rel_err(x, f64["solve_p0_it5"]) < 1e-8
    kn = zo.compute_kn(T64, f64["v"], maxiter_cg=20, tol=1e-8)
    if name in CLAMPED:
        assert rel_err(kn, f64["kn_it20"]) <= chaotic_bound(name, "f64", "kn_it20"), rel_err(kn, f64["kn_it20"])
    else:
        assert rel_err(kn, f64["kn_it20"]) < 1e-8


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_gram_solve_config1(tag):
    fx = load("G1", tag)
    g = fx["grid0"]
    kf = lambda x, y: zo.kernel_eval("matern", x, y, (1., .1), nu=2.5)
    vec = fx["vec"]
    for pre in (0, 1):
        for rt in (0, 1):
            for mi in (1, 5, 20):
                key = f"gram_p{pre}_rt{rt}_it{mi}"
                its = []
                res = zo.gram_solve([g], kf, vec, maxiter=mi, do_precond=bool(pre), tol=1e-10,
                                    callback=lambda n, x: its.append(n), mult_RT=bool(rt))
                assert res.shape == fx[key].shape
                if tag == "f64":
                    assert rel_err(res, fx[key]) < 1e-6, key
                    assert len(its) == int(fx[key + "_ncb"]), key


def test_compute_kn_model():
    fx = load("G5", "f64")
    grids = [fx["grid0"], fx["grid1"]]
    kf = lambda x, y: zo.kernel_eval("matern", x, y, (1., .1), nu=1.5)
    Knm = kf(fx["xobs"], zo.grid_points(grids))
    assert rel_err(Knm, fx["Knm"]) < 1e-12
    T = zo.ToeplitzOracle(zo.toeplitz_column(grids, kf, 1e-3), (20, 20))
    kn = zo.compute_kn(T, fx["Knm"], maxiter_cg=20, tol=1e-8)
    assert rel_err(kn, fx["kn"]) < 1e-8
