"""ToeplitzMatmul + gram_solve (`ziggy/misc/toeplitz_expanded.py:17-250`) on libhipgp.

ToeplitzMatmul is the older twin of ToeplitzTensor: NO nugget on the column
(`toeplitz_expanded.py:242-250`), multiply types "gram" | "RTv" | "Rv" | "circ_inv"
(`:139-189`).  gram_solve runs conj_grad's column-layout recurrence (`cg.py:5-41`) on vec^T (M, bsz) as the
reference does; its K / C^-1 operators are ColumnOp objects, so conj_grad runs the whole solve as
hgp_pcg_solve(LAYOUT_COLS) and the callback sees the (M, bsz) iterate.
"""
import numpy as np
import torch
from torch import nn

from hipgp_amd import _lib
from hipgp_amd.plan import ToeplitzPlan
from hipgp_amd.ziggy.misc.cg import ColumnOp, conj_grad

_OPS = {"gram": _lib.OP_K, "RTv": _lib.OP_RT, "Rv": _lib.OP_R, "circ_inv": _lib.OP_CINV}


def gram_solve(xgrids, kernel_fun, vec, K_matmul=None, maxiter=20, do_precond=True,
               tol=1e-10, callback=None, mult_RT=True):
    """R^T Kuu^{-1} vec^T (mult_RT) or Kuu^{-1} vec^T, vec (bsz, M)  (`:17-58`)."""
    assert len(vec.shape) == 2
    if K_matmul is None:
        K_matmul = ToeplitzMatmul(xgrids, kernel_fun, batch_shape=vec.shape[:-1])
    else:
        K_matmul.set_batch_shape(vec.shape[:-1])
    Kmul = ColumnOp(K_matmul._plan, _lib.OP_K)
    precond = ColumnOp(K_matmul._plan, _lib.OP_CINV) if do_precond else None
    # column layout as the reference (`:46-53`): one fused hgp_pcg_solve(LAYOUT_COLS)
    d = conj_grad(Kmul, vec.t(), precond=precond, maxiter=maxiter, tol=tol, callback=callback)  # (M, bsz)
    if mult_RT:
        return K_matmul(d.t(), multiply_type="RTv")
    return d.t()


class ToeplitzMatmul(nn.Module):
    def __init__(self, xgrids, kernel, batch_shape=None):
        super().__init__()
        self.device = xgrids[0].device
        self.dims = tuple(len(xg) for xg in xgrids)
        self.ndim = len(self.dims)
        self.M = np.prod(self.dims)
        self.xgrids = xgrids
        self.K = self.toeplitz_gram(xgrids, kernel)
        self._plan = ToeplitzPlan(self.dims, dtype=self.K.dtype, device=self.device)
        self._plan.set_column(self.K.reshape(-1), jitter=0.0, clamp_min=1e-6)
        self.res_idx = [slice(None)] + [slice(0, d, 1) for d in self.dims] + [0]
        self.Cc_shape = tuple(self._plan.ndims) + (2,)
        if batch_shape is not None:
            self.batch_shape = batch_shape
            self.cvec_shape = tuple(batch_shape) + self.Cc_shape

    def set_batch_shape(self, batch_shape):
        self.batch_shape = batch_shape
        self.cvec_shape = tuple(batch_shape) + self.Cc_shape

    def forward(self, vec, multiply_type="gram"):
        if multiply_type not in _OPS:
            raise NotImplementedError("gram|RTv|Rv|circ_inv")
        return self._plan.apply(_OPS[multiply_type], vec.reshape(vec.shape[0], -1))

    def circulant_embed(self, Ktoe):
        for d in range(len(Ktoe.shape)):
            Krev = torch.flip(Ktoe, dims=(d,))
            idx = tuple([slice(None)] * d + [slice(1, -1, 1)])
            Ktoe = torch.cat([Ktoe, Krev[idx]], dim=d)
        return Ktoe

    @property
    def C(self):
        return self.circulant_embed(self.K)

    def _pair(self, which):
        re = self._plan.spectrum(which)
        return torch.stack([re, torch.zeros_like(re)], dim=-1)

    @property
    def D(self):
        return self._pair(_lib.SPEC_D)

    @property
    def D_sqrt(self):
        return self._pair(_lib.SPEC_DSQRT)

    @property
    def Di(self):
        return self._pair(_lib.SPEC_DI)

    def toeplitz_gram(self, xgrids, kernel):
        """first row, no nugget (`toeplitz_expanded.py:242-250`)."""
        dims = [len(xg) for xg in xgrids]
        xxs = torch.meshgrid(*xgrids, indexing="ij")
        xs = torch.stack([x.reshape(-1) for x in xxs], dim=-1)
        Krow = kernel(xs[0][None, :], xs)
        return Krow.view(dims)
