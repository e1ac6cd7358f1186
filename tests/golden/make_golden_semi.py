"""Golden vectors for the line-integral (semi-integrated) cross covariance, SURVEY §8(f)
row 2, produced by running the *reference* `ziggy` kernels in THIS container (same
in-memory import shim as make_golden.py; no reference file copied or modified).

Per case (G8 3-D 6x5x4, G9 2-D 7x6) and dtype:
  * `SqExp.k_semi` (analytic, `kernels.py:80-85,223-237`) through `_make_grams`' transpose;
  * `Kernel.k_semi_mc` (`kernels.py:19-39`) for SqExp, Matern 1/2, 3/2, 5/2 and Gneiting with
    npts in {1, 10}, under a fixed torch seed; the single torch.rand(1) draw it consumes is
    recorded as `u_*` so the build can be handed the same offset;
  * `k_doubly_diag` (`kernels.py:168-220`): the interpolation table and its values at the
    observations (one at the origin: index -1 wraps) and beyond dmax.

Usage:  python tests/golden/make_golden_semi.py     (writes tests/golden/G8, G9, G10 *.npz)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, _np, import_reference  # noqa: E402

KERNELS = (("sqexp", None), ("matern", .5), ("matern", 1.5), ("matern", 2.5), ("gneiting", 1.))


def _kern(zk, kind, nu, dtype):
    if kind == "sqexp":
        return zk.SqExp(dtype=dtype)
    if kind == "matern":
        return zk.Matern(nu=nu, dtype=dtype)
    return zk.Gneiting(alpha=nu, dtype=dtype)


def gen_case(zk, dtype, tag, name, dims, lo, hi, nobs, params, seed):
    rs = np.random.RandomState(seed)
    xgrids = [torch.linspace(lo[d], hi[d], dims[d], dtype=dtype) for d in range(len(dims))]
    mesh = torch.meshgrid(*xgrids, indexing="ij")
    xinduce = torch.stack([g.reshape(-1) for g in mesh], dim=-1)
    # integrated observations: segment end points (the line runs from the origin)
    xo = rs.uniform(-1, 1, size=(nobs, len(dims))) * np.array(hi) * 1.5
    xo[0] = 0.                          # |x| = 0: zero integral, interpolation index -1
    xo[1] = np.array(hi) * 40.          # far beyond dmax * ell: interpolation extrapolates
    x = torch.tensor(xo, dtype=dtype)
    out = {f"grid{d}": _np(g) for d, g in enumerate(xgrids)}
    out["x"] = _np(x)
    out["params"] = np.array(params)
    for kind, nu in KERNELS:
        kern = _kern(zk, kind, nu, dtype)
        key = kind if nu is None else f"{kind}{nu}"
        if kind == "sqexp":
            out[f"semi_{key}"] = _np(kern.k_semi(xinduce, x, params).transpose(0, 1))
        for npts in (1, 10):
            torch.manual_seed(seed + npts)
            u = torch.rand(1, dtype=dtype)
            torch.manual_seed(seed + npts)
            out[f"mc_{key}_n{npts}"] = _np(kern.k_semi_mc(xinduce, x, params, npts=npts).transpose(0, 1))
            out[f"u_{key}_n{npts}"] = _np(u)
        di = kern.diag_interp
        out[f"dd_grid_{key}"] = _np(di.distance_grid)
        out[f"dd_knn_{key}"] = _np(di.knn)
        out[f"dd_slopes_{key}"] = _np(di.slopes)
        out[f"dd_{key}"] = _np(kern.k_doubly_diag(x, params))
    np.savez_compressed(os.path.join(OUT, f"{name}_{tag}.npz"), **out)


def gen_model(zk, hg, dtype, tag):
    """G10: MeanFieldToeplitzGP on a 3-D 8x6x5 grid over [-.25, .25]^3 (no clamped embedding
    eigenvalue, so kn is pinned tightly), SqExp (1, .1), 40 integrated observations, analytic
    Knm: elbo_and_grad (`hipgp.py:194-276` with `svi_gp.py:55-69`)."""
    torch.manual_seed(0)
    rs = np.random.RandomState(10)
    kern = zk.SqExp(dtype=dtype)
    lo, hi = (-.25, -.25, -.25), (.25, .25, .25)
    xgrids = [torch.linspace(lo[d], hi[d], m, dtype=dtype) for d, m in enumerate((8, 6, 5))]
    mod = hg.MeanFieldToeplitzGP(kern, xgrids, num_obs=40, sig2_init=1., ell_init=.1,
                                 noise2_init=.01, learn_kernel=False, dtype=dtype)
    x = torch.tensor(rs.uniform(-1, 1, size=(40, 3)) * np.array(hi), dtype=dtype)
    y = torch.tensor(rs.randn(40, 1), dtype=dtype)
    Knm, Knn = mod._make_grams(x, integrated_obs=True, semi_integrated_estimator="analytic")
    kn = mod.compute_kn(Knm, maxiter_cg=20)
    out = {f"grid{d}": _np(g) for d, g in enumerate(xgrids)}
    out.update(x=_np(x), y=_np(y), Knm=_np(Knm), Knn_diag=_np(Knn), kn=_np(kn),
               theta1=_np(mod.global_theta1), theta2=_np(mod.global_theta2))
    elbo = mod.elbo_and_grad(x, y, maxiter_cg=20, integrated_obs=True, semi_integrated_estimator="analytic")
    out["elbo"] = np.array(float(elbo))
    out["theta1_grad"] = _np(mod.global_theta1.grad)
    out["theta2_grad"] = _np(mod.global_theta2.grad)
    np.savez_compressed(os.path.join(OUT, f"G10_{tag}.npz"), **out)


def main():
    zk, tt, te, cg, hg = import_reference()
    torch.set_num_threads(8)
    for dtype, tag in ((torch.float64, "f64"), (torch.float32, "f32")):
        # G8: 3-D dust-like box (`run_domain_experiment.py:77-82` extents), Matern/SqExp (.1, .1)
        if sys.argv[1:] == ["model"]:
            gen_model(zk, hg, dtype, tag)
            continue
        gen_case(zk, dtype, tag, "G8", (6, 5, 4), (-.25, -.25, -.05), (.25, .25, .05), 24, (1., .1), 8)
        # G9: 2-D
        gen_case(zk, dtype, tag, "G9", (7, 6), (-1., -1.), (1., 1.), 16, (.7, .3), 9)
        gen_model(zk, hg, dtype, tag)
        print("wrote", tag)


if __name__ == "__main__":
    main()
