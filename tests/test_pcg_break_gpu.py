"""The device break test of the fused PCG (cg.py:69-71) against the same solve without it.

With the preconditioner the fused iteration applies x += alpha p in the C^-1 r pass
(hgp_rows.hpp EPI_XP), so a break right after an iteration's r update is finished by that
pass alone.  A solve that breaks at iteration k must therefore return exactly the iterate of
the same solve stopped by maxiter = k with the break disabled (tol < 0): same kernels, same
arithmetic, bit for bit -- 2-D and 3-D, fp32 and fp64, in one call (hgp_pcg_solve) and
stepwise (hgp_pcg_step)."""
import numpy as np
import pytest
import torch

from oracle import ziggy_oracle as zo

pytestmark = pytest.mark.gpu

CASES = {"2d_f32": ((128, 96), torch.float32), "2d_f64": ((96, 80), torch.float64),
         "3d_f32": ((32, 24, 20), torch.float32), "3d_f64": ((24, 20, 16), torch.float64),
         "2d_C2_f32": ((1024, 1024), torch.float32),
         # full BASELINE sizes: C5's 3-D grid (256-plane folds, k_cg_alpha) and C4's 4096-point rows
         "3d_C5_f32": ((256, 256, 128), torch.float32), "2d_C4_f32": ((4096, 4096), torch.float32)}


def _plan(dims, dt):
    from hipgp_amd.plan import ToeplitzPlan
    grids = [np.linspace(-1, 1, m) for m in dims]
    col = zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., .1), nu=1.5), 0.05)
    P = ToeplitzPlan(dims, dt, "cuda")
    P.set_column(torch.tensor(col, device="cuda", dtype=dt))
    return P


@pytest.mark.parametrize("case", sorted(CASES))
def test_break_equals_maxiter_stop(case):
    dims, dt = CASES[case]
    P = _plan(dims, dt)
    g = torch.Generator(device="cuda").manual_seed(5)
    b = torch.randn(4, int(np.prod(dims)), device="cuda", generator=g, dtype=torch.float64).to(dt)
    # a tolerance that every RHS meets only after a few iterations
    x20, it20 = P.pcg(b, 20, -1.0, precond=True, return_iters=True)
    assert it20 == 20
    from hipgp_amd import _lib
    r = b.double() - P.apply(_lib.OP_K, x20).double()
    tol = float(torch.linalg.norm(r, dim=1).max()) * 30.0
    xb, k = P.pcg(b, 200, tol, precond=True, return_iters=True)
    assert 1 <= k < 20, k
    xk, itk = P.pcg(b, k, -1.0, precond=True, return_iters=True)
    assert itk == k
    assert torch.equal(xb, xk), float((xb - xk).abs().max())
    # the stepwise form (callback path): converged flag after step k, same iterate
    seen = []
    xs = P.pcg_steps(b, 200, tol, precond=True, callback=lambda n, x: seen.append(n))
    assert len(seen) == k - 1, (len(seen), k)   # callback after every step that did not break
    assert torch.equal(xs, xk)
