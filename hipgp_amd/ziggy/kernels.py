"""Stationary kernels: the Toeplitz first row (hot-path row a1) and the line-integral
("semi-integrated") observation covariances.

Mirrors `ziggy/kernels.py` forward/diag of SqExp (:64-93), Gneiting (:96-128) and Matern
(:131-165) as torch modules, evaluated on whatever device the inputs live on, plus
`k_semi_mc` (:19-39), `SqExp.k_semi` (:80-85, 223-237) and the doubly-integrated diagonal
interpolator (:168-220).  On a gridded model the line-integral Knm is produced by the fused
HIP kernels of `hipgp_amd.kuf` (`ToeplitzInducingGP._make_grams`); the methods here evaluate
the same formulas for arbitrary point sets.  The doubly-integrated diagonal always runs through
`hgp_knn_doubly_diag`.
"""
import numpy as np
import torch
from torch import nn


def _np_kernel(kernel, x, y):
    """Scalar kernel value at params (1, 1) for the diagonal table, evaluated in NumPy in the
    kernel's dtype on float32-rounded inputs (the reference's integrand goes through
    `torch.Tensor(x).to(dtype)`, `kernels.py:180-183`)."""
    dt = np.float64 if kernel.dtype == torch.float64 else np.float32
    d = np.float32(x).astype(dt) - np.float32(y).astype(dt)
    if isinstance(kernel, SqExp):
        return float(np.exp(-np.sum(d * d) / dt(2)))
    if isinstance(kernel, Matern):
        sq = np.sum(d * d)
        r = np.sqrt(sq)
        if kernel.nu == .5:
            return float(np.exp(-r))
        if kernel.nu == 1.5:
            dp = dt(np.sqrt(3)) * r
            return float((1 + dp) * np.exp(-dp))
        dp = dt(np.sqrt(5)) * r
        return float((1 + dp + dt(5. / 3.) * sq) * np.exp(-dp))
    t = np.sqrt(np.sum(d * d))
    c = (1 - t) * np.cos(dt(np.pi) * t) + dt(1 / np.pi) * np.sin(dt(np.pi) * t)
    c = (1 + t ** kernel.alpha) ** (-3) * c
    return 0. if t > 1. else float(c)


class KernelDoublyDiagInterpolator(nn.Module):
    """`kernels.py:168-220`: knn(d) = |x|^2 int_0^1 int_0^1 k(a x, a' x) da da' at x = (d, 0)
    on N points of [0, dmax] (scipy dblquad, the reference's tolerances, `kernels.py:266-289`),
    stored as float32 then cast (`torch.Tensor(...).to(dtype)`); forward interpolates linearly
    in |x / ell| on the device (`hgp_knn_doubly_diag`)."""

    def __init__(self, kernel, N=50, dmax=5, dtype=None):
        super().__init__()
        from scipy import integrate
        dtype = kernel.dtype if dtype is None else dtype
        dgrid = np.linspace(0, dmax, N)
        knn = np.zeros(N)
        for n, dn in enumerate(dgrid):
            xn = np.array([dn, 0.])
            f = lambda a, ap: _np_kernel(kernel, a * xn, ap * xn)
            res = integrate.dblquad(f, a=0, b=1, gfun=lambda a: 0, hfun=lambda b: 1,
                                    epsrel=1.49e-5, epsabs=1.49e-1)
            knn[n] = res[0] * (dn * dn)
        slopes = (knn[1:] - knn[:-1]) / (dgrid[1:] - dgrid[:-1])
        slopes = np.concatenate([slopes, [slopes[-1]]])
        self.distance_grid = torch.Tensor(dgrid).to(dtype)
        self.slopes = torch.Tensor(slopes).to(dtype)
        self.knn = torch.Tensor(knn).to(dtype)
        self._dev = {}

    def table(self, device, dtype):
        key = (str(device), dtype)
        if key not in self._dev:
            self._dev[key] = torch.stack([self.distance_grid, self.knn, self.slopes]).to(device=device, dtype=dtype)
        return self._dev[key]

    def forward(self, x, params):
        from hipgp_amd.kuf import knn_doubly_diag
        return knn_doubly_diag(self.table(x.device, x.dtype), x, params)


class Kernel(nn.Module):
    def __init__(self):
        super().__init__()

    @property
    def diag_interp(self):
        """Built on first use (the reference builds it in every kernel's __init__,
        `kernels.py:70-71,104-105,140-141`; the table does not depend on params)."""
        di = self.__dict__.get("_diag_interp")
        if di is None:
            di = KernelDoublyDiagInterpolator(self, N=getattr(self, "Ndiag", 50), dmax=getattr(self, "dmax", 5))
            self.__dict__["_diag_interp"] = di
        return di

    def k_semi(self, xpoint, xintegrated, params):
        raise NotImplementedError

    def k_semi_mc(self, xpoint, xintegrated, params, npts=5, u=None):
        """`kernels.py:19-39`: (Np, Ni) = |x_i| mean_a k(xpoint_p, alpha_a x_i).  `u`: the offset
        draw to use instead of the reference's own torch.rand(1) (sharded fits share rank 0's)."""
        Np, D = xpoint.shape
        Ni, D = xintegrated.shape
        delta = 1. / npts
        if u is None:
            u = torch.rand(1, dtype=self.dtype, device=xpoint.device)
        alphas = torch.arange(npts, dtype=self.dtype, device=xpoint.device) / npts + \
            u.to(device=xpoint.device, dtype=self.dtype).reshape(1) * delta
        xgrid = xintegrated[:, None, :] * alphas[None, :, None]
        Kpis = self.forward(xpoint, xgrid.reshape(-1, D), params=params).reshape(Np, Ni, npts)
        dists = xintegrated.pow(2.).sum(dim=-1).sqrt()
        return torch.mean(Kpis, dim=-1) * dists[None, :]

    def k_semi_num(self, xpoint, xintegrated, params):
        raise NotImplementedError("scipy-quad validation estimator of the reference (kernels.py:41-50): "
                                  "not part of the device path")

    def k_doubly_diag(self, x, params):
        return self.diag_interp(x, params)


class SqExp(Kernel):
    """`kernels.py:64-93`."""

    def __init__(self, dtype=torch.double, Ndiag=50, dmax=5):
        super().__init__()
        self.dtype = dtype
        self.Ndiag, self.dmax = Ndiag, dmax
        self.has_k_semi = True

    def forward(self, x, y, params):
        assert x.shape[-1] == y.shape[-1]
        assert x.ndimension() == 2 and y.ndimension() == 2
        sig2, ell = params
        sqdist = torch.sum(((x[:, None, :] - y[None, :, :]) / ell) ** 2, dim=-1)
        return sig2 * torch.exp(-sqdist / 2)

    def diag(self, x, params):
        sig2, ell = params
        return sig2 * torch.ones(x.shape[0], dtype=self.dtype, device=x.device)

    def k_semi(self, xpoint, xintegrated, params):
        """`kernels.py:80-85`: (Np, Ni) analytic line integral for arbitrary points."""
        sig2, ell = params
        D = xpoint.shape[1]
        Sinv = (1. / (ell ** 2)) * torch.eye(D, dtype=self.dtype, device=xpoint.device)
        return semi_integrated_sqe(xintegrated, xpoint, sig2, Sinv).transpose(0, 1)


sqrt2pi = np.sqrt(2 * np.pi)


def semi_integrated_sqe(xintegrated, x, sig2, Sinv):
    """`kernels.py:223-237` (integrates over the FIRST argument); (Ni, Np)."""
    xdists = torch.sqrt(torch.sum(xintegrated * xintegrated, dim=-1))
    a = torch.sum(torch.matmul(xintegrated, Sinv) * xintegrated, dim=-1)
    xint_Si = torch.matmul(xintegrated, Sinv)
    b = xint_Si @ x.transpose(0, 1)
    c = torch.sum(torch.matmul(x, Sinv) * x, dim=-1)
    scale = torch.sqrt(1 / a[:, None])
    loc = b / a[:, None]
    coef = sig2 * torch.exp((b ** 2) / (2 * a[:, None]) - c / 2) * sqrt2pi * scale
    sq2 = np.sqrt(2)
    ca = .5 * (1. + torch.erf((1 - loc) / (scale * sq2)))
    cb = .5 * (1. + torch.erf((0 - loc) / (scale * sq2)))
    return coef * (ca - cb) * xdists[:, None]


class Gneiting(Kernel):
    """`kernels.py:96-128`."""

    def __init__(self, alpha=1., length_scale=1., dtype=torch.double, Ndiag=50, dmax=5.):
        super().__init__()
        self.dtype = dtype
        self.alpha = alpha
        self.length_scale = length_scale
        self.anisotropic = False
        self.Ndiag, self.dmax = Ndiag, dmax
        self.has_k_semi = False

    def forward(self, x, y, params):
        sig2, ell = params
        t = torch.sqrt(torch.sum(((x[:, None, :] - y[None, :, :]) / ell) ** 2, dim=-1))
        cterms = (1 - t) * torch.cos(np.pi * t) + (1 / np.pi) * torch.sin(np.pi * t)
        cij = (1 + t ** self.alpha) ** (-3) * cterms
        cij[t > 1.] = 0.
        return sig2 * cij

    def diag(self, x, params):
        sig2, ell = params
        return sig2 * torch.ones(x.shape[0], dtype=self.dtype, device=x.device)


class Matern(Kernel):
    """`kernels.py:131-165` (nu in {0.5, 1.5, 2.5})."""

    def __init__(self, nu=0.5, length_scale=1., dtype=torch.double, Ndiag=50, dmax=5.):
        super().__init__()
        if nu not in {0.5, 1.5, 2.5}:
            raise RuntimeError("nu expected to be 0.5, 1.5, or 2.5")
        self.nu = nu
        self.dtype = dtype
        self.length_scale = length_scale
        self.anisotropic = False
        self.Ndiag, self.dmax = Ndiag, dmax
        self.has_k_semi = False

    def forward(self, x, y, params):
        assert x.shape[-1] == y.shape[-1]
        sig2, ell = params
        sqdist = torch.sum((x[:, None, :] - y[None, :, :]) ** 2, dim=-1)
        if self.nu == .5:
            kmat = torch.exp(-torch.sqrt(sqdist) / ell)
        elif self.nu == 1.5:
            dp = np.sqrt(3) * torch.sqrt(sqdist) / ell
            kmat = (1 + dp) * torch.exp(-dp)
        else:
            dp = np.sqrt(5) * torch.sqrt(sqdist) / ell
            kmat = (1 + dp + (5. / 3.) * sqdist / (ell ** 2)) * torch.exp(-dp)
        return sig2 * kmat

    def diag(self, x, params):
        sig2, ell = params
        return sig2 * x.new_ones(x.shape[0])
