"""Backward golden cases (tests/golden/make_golden_grad.py, made by running the reference):
name -> (kernel kind, nu, (sig2, ell)); grids linspace(-1, 1, m), jitter 1e-3, PCG maxiter 30, tol 1e-10."""
GRAD_CASES = {
    "G13": ("matern", 2.5, (1., .3)),
    "G14": ("sqexp", None, (1., .4)),
    "G15": ("matern", 1.5, (1., .6)),
}
GRAD_MAXITER, GRAD_TOL = 30, 1e-10
