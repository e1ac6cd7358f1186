"""The two passes of the mean-field statistics apart (hgp_meanfield_rowdots / hgp_meanfield_cols,
grid-block sharding: kn held in column slabs) against the torch expression of the same sums
(`hipgp.py:234-250`, a_n of `hipgp.py:370-414`), and MeanFieldToeplitzGP.batch_stats_slab over a
split of the columns -- summed as the ranks' all-reduce would -- against batch_stats of the whole
kn (one process, no collective: `reduce` sums the slabs' dots here)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dt,tol", [(torch.float64, 1e-12), (torch.float32, 2e-5)])
@pytest.mark.parametrize("B,Mp", [(1, 1), (7, 1000), (33, 70001)])
def test_rowdots_and_cols_vs_torch(dt, tol, B, Mp):
    from hipgp_amd import _lib
    g = torch.Generator(device=DEV).manual_seed(B + Mp)
    kn = torch.randn(B, Mp, device=DEV, dtype=dt, generator=g)
    qm = torch.randn(Mp, device=DEV, dtype=dt, generator=g)
    qS = torch.rand(Mp, device=DEV, dtype=dt, generator=g)
    iv = torch.rand(B, device=DEV, dtype=dt, generator=g) + .5
    bd = torch.randn(B, device=DEV, dtype=dt, generator=g)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    dots = torch.empty(B, 3, device=DEV, dtype=dt)
    _lib.check(_lib.lib().hgp_meanfield_rowdots(_lib.dtype_code(dt), p(kn), B, Mp, p(qm), p(qS), p(dots),
                                                _lib.stream_ptr(kn.device)))
    k64 = kn.double()
    ref = torch.stack([k64 @ qm.double(), (k64 * k64).sum(1), (k64 * k64) @ qS.double()], 1)
    assert float((dots.double() - ref).abs().max() / ref.abs().max()) < tol
    lam = torch.empty(Mp, device=DEV, dtype=dt)
    dm = torch.empty(Mp, device=DEV, dtype=dt)
    _lib.check(_lib.lib().hgp_meanfield_cols(_lib.dtype_code(dt), p(kn), B, Mp, p(iv), p(bd), p(lam), p(dm),
                                             _lib.stream_ptr(kn.device)))
    lref = (iv.double()[:, None] * k64 * k64).sum(0)
    dref = -(bd.double()[:, None] * k64).sum(0)
    assert float((lam.double() - lref).abs().max() / lref.abs().max()) < tol
    assert float((dm.double() - dref).abs().max() / dref.abs().max()) < tol


def test_rowdots_cols_empty_and_refused():
    from hipgp_amd import _lib
    L = _lib.lib()
    assert L.hgp_meanfield_rowdots(_lib.dtype_code(torch.float64), None, 0, 0, None, None, None, None) == 0
    assert L.hgp_meanfield_cols(0, None, 3, 0, None, None, None, None, None) == 0
    assert L.hgp_meanfield_rowdots(9, None, 1, 1, None, None, None, None) != 0


@pytest.mark.parametrize("noise", ["per_obs", "shared"])
def test_batch_stats_slab_sums_to_batch_stats(noise):
    """batch_stats_slab over three column slabs (uneven), their dots summed (what the ranks'
    all-reduce does) and their M'-vectors summed (allreduce_stats), equals batch_stats (fp64)."""
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    dt = torch.float64
    grids = [torch.linspace(-1, 1, 9, dtype=dt), torch.linspace(-1, 1, 7, dtype=dt)]
    mod = hg.MeanFieldToeplitzGP(zk.Matern(nu=1.5, dtype=dt), grids, num_obs=100, sig2_init=1., ell_init=.3,
                                 learn_kernel=False, dtype=dt).cuda_params(0)
    g = torch.Generator(device=DEV).manual_seed(3)
    with torch.no_grad():
        mod.global_theta1.copy_(torch.randn(mod.Mprime, 1, device=DEV, dtype=dt, generator=g))
    B, Mp = 11, mod.Mprime
    kn = torch.randn(B, Mp, device=DEV, dtype=dt, generator=g)
    y = torch.randn(B, 1, device=DEV, dtype=dt, generator=g)
    knn = torch.rand(B, device=DEV, dtype=dt, generator=g) + 2
    s = torch.rand(B, 1, device=DEV, dtype=dt, generator=g) * .2 + .05 if noise == "per_obs" else None
    with torch.no_grad():
        full = mod.batch_stats(kn, y, knn, s)
        cuts = [0, Mp // 3 + 5, 2 * Mp // 3, Mp]
        # pass 1 on every slab, the dots summed over the slabs (what the ranks' all-reduce does) ...
        total = torch.zeros(B, 3, device=DEV, dtype=dt)
        for r in range(3):
            j0, j1 = cuts[r], cuts[r + 1]
            mod.batch_stats_slab(kn[:, j0:j1].contiguous(), j0, y, knn, s, reduce=lambda t: total.add_(t), lead=False)
        # ... then each slab's statistics with the summed dots
        stats = []
        for r in range(3):
            j0, j1 = cuts[r], cuts[r + 1]
            stats.append(mod.batch_stats_slab(kn[:, j0:j1].contiguous(), j0, y, knn, s,
                                              reduce=lambda t: t.copy_(total), lead=r == 0))
    lam = sum(st["lam_sum"] for st in stats)
    dm = sum(st["dm_sum"] for st in stats)
    an = sum(float(st["an_sum"]) for st in stats)
    n = sum(st["n"] for st in stats)
    assert n == B
    assert float((lam - full["lam_sum"]).abs().max() / full["lam_sum"].abs().max()) < 1e-12
    assert float((dm - full["dm_sum"]).abs().max() / full["dm_sum"].abs().max()) < 1e-12
    assert abs(an - float(full["an_sum"])) < 1e-10 * abs(float(full["an_sum"]))
