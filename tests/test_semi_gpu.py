"""Line-integral (semi-integrated) cross covariance on the GPU, SURVEY §8(f) row 2:
hgp_kuf_semi_mc / hgp_kuf_semi_sqexp / hgp_knn_doubly_diag against the reference's own
outputs (tests/golden/make_golden_semi.py fixtures G8 3-D, G9 2-D; the MC offset draw the
reference consumed is handed over explicitly) and, at the config-5 grid size, against the
same formulas evaluated by broadcasting on the device."""
import numpy as np
import pytest
import torch

from golden_cases import SEMI_CASES, SEMI_KERNELS, load, grids_of, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _kern(key, dtype):
    import ziggy.kernels as zk
    kind, nu = SEMI_KERNELS[key]
    if kind == "sqexp":
        return zk.SqExp(dtype=dtype)
    if kind == "matern":
        return zk.Matern(nu=nu, dtype=dtype)
    return zk.Gneiting(alpha=nu, dtype=dtype)


def _dt(tag):
    return torch.float64 if tag == "f64" else torch.float32


@pytest.mark.parametrize("name", sorted(SEMI_CASES))
@pytest.mark.parametrize("tag", ["f64", "f32"])
@pytest.mark.parametrize("npts", [1, 10])
def test_semi_mc_reference(name, tag, npts):
    from hipgp_amd.kuf import kuf_semi_mc
    fx = load(name, tag)
    dt = _dt(tag)
    grids = [torch.tensor(g, device=DEV) for g in grids_of(fx)]
    x = torch.tensor(fx["x"], device=DEV)
    params = SEMI_CASES[name]
    for key in SEMI_KERNELS:
        u = torch.tensor(fx[f"u_{key}_n{npts}"])
        out = kuf_semi_mc(_kern(key, dt), grids, x, params, npts, u=u)
        assert out is not None and out.dtype == dt
        tol = 1e-13 if tag == "f64" else 3e-6
        assert rel_err(out.cpu().numpy(), fx[f"mc_{key}_n{npts}"]) < tol, key


@pytest.mark.parametrize("name", sorted(SEMI_CASES))
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_semi_sqexp_reference(name, tag):
    from hipgp_amd.kuf import kuf_semi_sqexp
    fx = load(name, tag)
    grids = [torch.tensor(g, device=DEV) for g in grids_of(fx)]
    out = kuf_semi_sqexp(_kern("sqexp", _dt(tag)), grids, torch.tensor(fx["x"], device=DEV), SEMI_CASES[name])
    # fp32: Phi(1) - Phi(0) cancels; error relative to the largest entry (see test_oracle_semi)
    assert rel_err(out.cpu().numpy(), fx["semi_sqexp"]) < (1e-12 if tag == "f64" else 2e-5)
    assert np.isnan(out[0].cpu().numpy()).all()          # zero-length segment: NaN as reference


@pytest.mark.parametrize("name", sorted(SEMI_CASES))
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_doubly_diag_reference(name, tag):
    from hipgp_amd.kuf import knn_doubly_diag
    fx = load(name, tag)
    x = torch.tensor(fx["x"], device=DEV)
    for key in SEMI_KERNELS:
        tab = torch.tensor(np.stack([fx[f"dd_grid_{key}"], fx[f"dd_knn_{key}"], fx[f"dd_slopes_{key}"]]))
        out = knn_doubly_diag(tab, x, SEMI_CASES[name])
        assert rel_err(out.cpu().numpy(), fx[f"dd_{key}"]) < (1e-13 if tag == "f64" else 1e-6), key
    # the kernel's own table (built here by dblquad) gives the same values
    out = _kern("matern1.5", _dt(tag)).k_doubly_diag(x, SEMI_CASES[name])
    assert rel_err(out.cpu().numpy(), fx["dd_matern1.5"]) < (1e-13 if tag == "f64" else 2e-6)


def test_model_integrated_grams_route():
    """_make_grams(integrated_obs=True) goes through the fused kernels and matches the
    kernel methods (broadcast formulas) on the same draw."""
    import ziggy.hipgp as hg
    dt = torch.float64
    k = _kern("matern2.5", dt)
    grids = [torch.linspace(-.25, .25, 9, dtype=dt), torch.linspace(-.25, .25, 7, dtype=dt),
             torch.linspace(-.05, .05, 5, dtype=dt)]
    mod = hg.MeanFieldToeplitzGP(k, grids, num_obs=32, sig2_init=1., ell_init=.1, noise2_init=.01,
                                 learn_kernel=False, dtype=dt).cuda_params(0)
    x = (torch.rand(12, 3, generator=torch.Generator().manual_seed(3), dtype=dt) - .5).to(DEV)
    torch.manual_seed(11)
    Knm, Knn = mod._make_grams(x, integrated_obs=True, semi_integrated_estimator="mc-biased",
                               semi_integrated_samps=10)
    torch.manual_seed(11)
    ref = k.k_semi_mc(mod.xinduce.to(DEV), x, mod.get_kernel_params(), npts=10).transpose(0, 1)
    assert rel_err(Knm.cpu().numpy(), ref.cpu().numpy()) < 1e-13
    assert Knn.shape == (12,)
    ks = _kern("sqexp", dt)
    mod2 = hg.MeanFieldToeplitzGP(ks, grids, num_obs=32, sig2_init=1., ell_init=.1, noise2_init=.01,
                                  learn_kernel=False, dtype=dt).cuda_params(0)
    Knm2, _ = mod2._make_grams(x, integrated_obs=True, semi_integrated_estimator="analytic")
    ref2 = ks.k_semi(mod2.xinduce.to(DEV), x, mod2.get_kernel_params()).transpose(0, 1)
    assert rel_err(Knm2.cpu().numpy(), ref2.cpu().numpy()) < 1e-12


def test_semi_mc_full_size_C5():
    """Config-5 grid 256 x 256 x 128, 200 integrated observations, npts 10, fp32: a sample of
    grid columns against the broadcast formula on the same offset draw."""
    from hipgp_amd.kuf import kuf_semi_mc
    dt = torch.float32
    k = _kern("matern2.5", dt)
    grids = [torch.linspace(-.25, .25, 256, device=DEV), torch.linspace(-.25, .25, 256, device=DEV),
             torch.linspace(-.05, .05, 128, device=DEV)]
    g = torch.Generator().manual_seed(4)
    x = ((torch.rand(200, 3, generator=g) - .5) * torch.tensor([.5, .5, .1])).to(DEV)
    u = torch.tensor([0.37])
    out = kuf_semi_mc(k, grids, x, (0.1, 0.1), 10, u=u)
    assert out.shape == (200, 256 * 256 * 128)
    assert torch.isfinite(out).all()
    cols = torch.randint(0, out.shape[1], (4096,), generator=g).to(DEV)
    i0, rem = cols // (256 * 128), cols % (256 * 128)
    pts = torch.stack([grids[0][i0], grids[1][rem // 128], grids[2][rem % 128]], dim=-1)
    alphas = torch.arange(10, dtype=dt, device=DEV) / 10 + u.to(DEV, dt) * (1. / 10)
    xg = (x[:, None, :] * alphas[None, :, None]).reshape(-1, 3)
    ref = (k.forward(pts, xg, params=(0.1, 0.1)).reshape(4096, 200, 10).mean(-1)
           * x.pow(2).sum(-1).sqrt()[None, :]).T
    assert rel_err(out[:, cols].cpu().numpy(), ref.cpu().numpy()) < 2e-6


def test_model_integrated_elbo_G10():
    """Reference MeanFieldToeplitzGP.elbo_and_grad with line-integral observations (analytic
    SqExp Knm, doubly-integrated Knn_diag) on a 3-D grid, fp64 (G10 fixture)."""
    import ziggy.hipgp as hg
    fx = load("G10", "f64")
    dt = torch.float64
    grids = [torch.tensor(fx[f"grid{d}"]) for d in range(3)]
    mod = hg.MeanFieldToeplitzGP(_kern("sqexp", dt), grids, num_obs=40, sig2_init=1., ell_init=.1,
                                 noise2_init=.01, learn_kernel=False, dtype=dt)
    with torch.no_grad():
        mod.global_theta1.copy_(torch.tensor(fx["theta1"]))
        mod.global_theta2.copy_(torch.tensor(fx["theta2"]))
    mod = mod.cuda_params(0)
    x = torch.tensor(fx["x"], device=DEV)
    y = torch.tensor(fx["y"], device=DEV)
    Knm, Knn = mod._make_grams(x, integrated_obs=True, semi_integrated_estimator="analytic")
    assert rel_err(Knm.cpu().numpy(), fx["Knm"]) < 1e-12
    assert rel_err(Knn.cpu().numpy(), fx["Knn_diag"]) < 1e-12
    elbo = mod.elbo_and_grad(x, y, maxiter_cg=20, integrated_obs=True, semi_integrated_estimator="analytic")
    assert abs(float(elbo) - float(fx["elbo"])) < 1e-8 * abs(float(fx["elbo"]))
    assert rel_err(mod.global_theta1.grad.cpu().numpy(), fx["theta1_grad"]) < 1e-7
    assert rel_err(mod.global_theta2.grad.cpu().numpy(), fx["theta2_grad"]) < 1e-7
