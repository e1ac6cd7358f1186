"""Stationary kernels used to generate the Toeplitz first row (hot-path row a1).

Mirrors `ziggy/kernels.py` forward/diag of SqExp (:64-93), Gneiting (:96-128) and Matern
(:131-165) as torch modules, evaluated on whatever device the inputs live on.  The
integrated-observation estimators (k_semi, k_semi_mc, doubly-integrated diagonal) are the
SURVEY §8(f) "next" rows and are not part of this round.
"""
import numpy as np
import torch
from torch import nn


class Kernel(nn.Module):
    def __init__(self):
        super().__init__()

    def k_semi(self, xpoint, xintegrated, params):
        raise NotImplementedError("line-integral Kuf is SURVEY §8(f) row 2 (not built yet)")

    def k_semi_mc(self, xpoint, xintegrated, params, npts=5):
        raise NotImplementedError("line-integral Kuf is SURVEY §8(f) row 2 (not built yet)")

    def k_doubly_diag(self, x, params):
        raise NotImplementedError("doubly-integrated diagonal is SURVEY §8(f) row 2")


class SqExp(Kernel):
    """`kernels.py:64-93`."""

    def __init__(self, dtype=torch.double, Ndiag=50, dmax=5):
        super().__init__()
        self.dtype = dtype
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


class Gneiting(Kernel):
    """`kernels.py:96-128`."""

    def __init__(self, alpha=1., length_scale=1., dtype=torch.double, Ndiag=50, dmax=5.):
        super().__init__()
        self.dtype = dtype
        self.alpha = alpha
        self.length_scale = length_scale
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
