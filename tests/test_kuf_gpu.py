"""Fused grid cross covariance (hgp_kuf_grid) against the broadcast
evaluation of the same kernels (`kernels.py:73-79, 145-158`, mirrored in ziggy.kernels) and
against the reference's own Knm (G5 fixture)."""
import numpy as np
import pytest
import torch

from golden_cases import load, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"

KERNELS = [("sqexp", None), ("matern", 0.5), ("matern", 1.5), ("matern", 2.5)]
GRIDS = [(300,), (64, 48), (17, 9, 5)]


def _kern(kind, nu, dtype):
    import ziggy.kernels as zk
    return zk.SqExp(dtype=dtype) if kind == "sqexp" else zk.Matern(nu=nu, dtype=dtype)


@pytest.mark.parametrize("kern", KERNELS, ids=lambda k: f"{k[0]}{k[1] or ''}")
@pytest.mark.parametrize("dims", GRIDS, ids=lambda d: "x".join(map(str, d)))
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32], ids=["f64", "f32"])
def test_kuf_matches_broadcast_kernel(kern, dims, dtype):
    from hipgp_amd.kuf import kuf_grid
    k = _kern(*kern, dtype)
    params = (1.3, 0.27)
    grids = [torch.linspace(-1, 1, m, dtype=dtype, device=DEV) for m in dims]
    g = torch.Generator(device="cpu").manual_seed(5)
    x = (torch.rand(37, len(dims), generator=g, dtype=dtype) * 2.4 - 1.2).to(DEV)
    mesh = torch.meshgrid(*grids, indexing="ij")
    xs = torch.stack([a.reshape(-1) for a in mesh], dim=-1)
    ref = k.forward(x, xs, params=params)
    out = kuf_grid(k, grids, x, params)
    assert out is not None and out.shape == ref.shape
    tol = 1e-13 if dtype == torch.float64 else 2e-6
    assert rel_err(out.cpu().numpy(), ref.cpu().numpy()) < tol


def test_kuf_reference_G5():
    """Knm of the reference's MeanFieldToeplitzGP._make_grams (svi_gp.py:72), fp64."""
    fx = load("G5", "f64")
    import ziggy.hipgp as hg
    k = _kern("matern", 1.5, torch.float64)
    grids = [torch.tensor(fx["grid0"]), torch.tensor(fx["grid1"])]
    mod = hg.MeanFieldToeplitzGP(k, grids, num_obs=64, sig2_init=1., ell_init=.1, noise2_init=.01,
                                 dtype=torch.float64).cuda_params(0)
    Knm, Knn = mod._make_grams(torch.tensor(fx["xobs"], device=DEV))
    assert rel_err(Knm.cpu().numpy(), fx["Knm"]) < 1e-12
    assert rel_err(Knn.cpu().numpy(), fx["Knn_diag"]) < 1e-12


def test_kuf_full_size_C2():
    """32 observations x the 1024^2 mesh (BASELINE C2), fp32, against the broadcast kernel."""
    from hipgp_amd.kuf import kuf_grid
    k = _kern("sqexp", None, torch.float32)
    grids = [torch.linspace(-1, 1, 1024, device=DEV) for _ in range(2)]
    x = (torch.rand(32, 2, generator=torch.Generator().manual_seed(1)) * 2 - 1).to(DEV)
    mesh = torch.meshgrid(*grids, indexing="ij")
    xs = torch.stack([a.reshape(-1) for a in mesh], dim=-1)
    ref = torch.cat([k.forward(x[i:i + 4], xs, params=(1.0, 0.01)) for i in range(0, 32, 4)])
    out = kuf_grid(k, grids, x, (1.0, 0.01))
    assert float((out - ref).abs().max()) <= 2e-6 * float(ref.abs().max())


def test_kuf_declines_when_grad_needed():
    from hipgp_amd.kuf import kuf_grid
    k = _kern("sqexp", None, torch.float32)
    grids = [torch.linspace(-1, 1, 8, device=DEV)] * 2
    ell = torch.tensor(0.3, device=DEV, requires_grad=True)
    assert kuf_grid(k, grids, torch.zeros(3, 2, device=DEV), (1.0, ell)) is None
