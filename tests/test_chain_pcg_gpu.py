"""The chained 2-D PCG iteration (HGP_CHAIN_PCG=1, off by default: measured slower, DESIGN §11
item 6) against the default fused iteration: K's row-inverse pass leaves C^-1's forward row
transform of the new r (EPI_RF) and C^-1 continues at its axis-0 pass.  The arithmetic of
`cg.py:63-78` is the same, so the iterates agree to rounding -- with and without the all-RHS
break firing (the path had no test)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _plan(dims, dt, chain):
    """A fresh plan (grids no other test uses, so nothing comes from the idle pool) with the
    chain switch read at creation."""
    from hipgp_amd.plan import ToeplitzPlan, release_pool
    from oracle import ziggy_oracle as zo
    release_pool()
    old = os.environ.get("HGP_CHAIN_PCG")
    os.environ["HGP_CHAIN_PCG"] = "1" if chain else "0"
    try:
        P = ToeplitzPlan(dims, dtype=dt, device="cuda")
    finally:
        if old is None:
            del os.environ["HGP_CHAIN_PCG"]
        else:
            os.environ["HGP_CHAIN_PCG"] = old
    grids = [np.linspace(-1, 1, m) for m in dims]
    col = zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., .3), nu=1.5), 1e-2)
    P.set_column(torch.tensor(col, dtype=dt, device="cuda"))
    return P


# 20 iterations: the two orders of the same arithmetic agree to ~1e-13 (fp64); run to the break
# (115 iterations on this problem) the Krylov recurrence amplifies that rounding to ~5e-6 -- the
# same iteration count and a converged true residual are what the break case pins
@pytest.mark.parametrize("dt,maxiter,tol,bound", [(torch.float64, 20, -1.0, 1e-12), (torch.float64, 500, 1.0, 1e-4),
                                                  (torch.float32, 20, -1.0, 1e-5)])
def test_chained_pcg_matches_default(dt, maxiter, tol, bound):
    dims = (300, 260)
    rs = np.random.RandomState(9)
    b = torch.tensor(rs.randn(5, dims[0] * dims[1]), dtype=dt, device="cuda")
    out = {}
    for chain in (False, True):
        P = _plan(dims, dt, chain)
        x, it = P.pcg(b, maxiter, tol, precond=True, return_iters=True)
        if tol > 0:     # the break's own test: every RHS's true residual below tol (to rounding)
            from hipgp_amd import _lib
            res = (P.apply(_lib.OP_K, x) - b).norm(dim=1)
            assert float(res.max()) < 1.05 * tol, (chain, res)
        out[chain] = (x.double().cpu().numpy(), it)
        del P
    (x0, it0), (x1, it1) = out[False], out[True]
    assert it0 == it1, (it0, it1)
    if tol > 0:
        assert it0 < maxiter          # the break fired
    rel = float(np.max(np.linalg.norm(x1 - x0, axis=1) / np.linalg.norm(x0, axis=1)))
    print("chained vs default PCG", dt, maxiter, tol, "iterations", it0, "rel", rel)
    assert rel <= bound, rel
