"""ToeplitzTensor — same constructor, methods and attributes as the reference
`ziggy/misc/toeplitz_tensor.py:7-169`, computed by the gfx950 kernels of libhipgp.so.

Operator map (reference line -> here):
  __init__ spectrum setup (:12-33)      -> ToeplitzPlan.set_column  (hgp_plan_set_column)
  _matmul_by_K     (:70-83)             -> HGP_OP_K
  _matmul_by_RT    (:85-97)             -> HGP_OP_RT
  _matmul_by_R     (:99-112)            -> HGP_OP_R
  _matmul_by_Cinv  (:114-125)           -> HGP_OP_CINV
  _solve / conj_grad2 (:54-68)          -> hgp_pcg_solve (device-side early-exit flag)
The spectrum attributes C, D, D_sqrt, Di, Di_sqrt are materialised lazily (they are
M'-sized and the operators never need them).

Autograd: in the reference every operator is torch arithmetic on D = clamp(Re FFT(embed(column)))
(`:20-31`), so gradients reach the vector AND the column (kernel hyper-parameters).  Here
`_ToeplitzOp` gives the same: vector gradient = the adjoint operator (K, C^-1 self-adjoint;
R <-> R^T), column gradient = hgp_plan_column_grad.  Without a grad-requiring input the
operators call the plan directly.
"""
import numpy as np
import torch
from torch.autograd import Function

from hipgp_amd import _lib
from hipgp_amd.plan import ToeplitzPlan
from hipgp_amd.ziggy.misc._inv_matmul import InvMatmul
from hipgp_amd.ziggy.misc.cg import conj_grad2


_ADJOINT = {_lib.OP_K: _lib.OP_K, _lib.OP_CINV: _lib.OP_CINV, _lib.OP_RT: _lib.OP_R, _lib.OP_R: _lib.OP_RT}


class _ToeplitzOp(Function):
    @staticmethod
    def forward(ctx, plan, op, column, vec):
        ctx.plan, ctx.op = plan, op
        ctx.save_for_backward(vec)
        return plan.apply(op, vec.detach())

    @staticmethod
    def backward(ctx, grad):
        (vec,) = ctx.saved_tensors
        grad = grad.contiguous()
        gcol = gvec = None
        if ctx.needs_input_grad[2]:
            gcol = ctx.plan.column_grad(ctx.op, vec.detach(), grad)
        if ctx.needs_input_grad[3]:
            gvec = ctx.plan.apply(_ADJOINT[ctx.op], grad)
        return None, None, gcol, gvec


class ToeplitzTensor:
    def __init__(self, xgrids, kernel, batch_shape=None, jitter_val=1e-3):
        self.column = self.toeplitz_gram(xgrids, kernel, jitter_val)
        self.device = xgrids[0].device
        self.dims = tuple(len(xg) for xg in xgrids)
        self.ndim = len(self.dims)
        self.M = np.prod(self.dims)
        self._plan = ToeplitzPlan(self.dims, dtype=self.column.dtype, device=self.device)
        # the column already carries the nugget (toeplitz_gram), so jitter=0 here
        self._plan.set_column(self.column, jitter=0.0, clamp_min=1e-6)
        self.res_idx = [slice(None)] + [slice(0, d, 1) for d in self.dims] + [0]
        self.Cc_shape = tuple(self._plan.ndims) + (2,)
        if batch_shape is not None:
            self.batch_shape = batch_shape
            self.cvec_shape = tuple(batch_shape) + self.Cc_shape

    # ---- reference API ---------------------------------------------------------------------
    def inv_matmul(self, right_tensor, do_precond=True, maxiter=20, tol=1e-8):
        """compute A^{-1}R, where self = A  (`toeplitz_tensor.py:47-52`)"""
        return InvMatmul.apply(self, self.column, right_tensor, do_precond, maxiter, tol)

    def _solve(self, vec, do_precond=True, maxiter=100, tol=1e-8, callback=None):
        """vec: (bsz, M) -> K^{-1} vec by PCG (`toeplitz_tensor.py:54-68`)."""
        assert len(vec.shape) == 2
        self.set_batch_shape(vec.shape[:-1])
        precond = self._matmul_by_Cinv if do_precond else None
        return conj_grad2(self._matmul_by_K, vec, precond=precond, maxiter=maxiter, tol=tol,
                          callback=callback)

    def _check_batch(self):
        # the reference needs batch_shape before any _matmul_by_* (it builds cvec_shape
        # from it, toeplitz_tensor.py:150): keep the same AttributeError behaviour.
        return self.cvec_shape

    def _op(self, op, vec):
        if torch.is_grad_enabled() and (vec.requires_grad or self.column.requires_grad):
            return _ToeplitzOp.apply(self._plan, op, self.column, vec)
        return self._plan.apply(op, vec)

    def _matmul_by_K(self, vec):
        self._check_batch()
        return self._op(_lib.OP_K, vec)

    def _matmul_by_RT(self, vec):
        self._check_batch()
        return self._op(_lib.OP_RT, vec)

    def _matmul_by_R(self, vec):
        self._check_batch()
        return self._op(_lib.OP_R, vec.reshape(vec.shape[0], -1))

    def _matmul_by_Cinv(self, vec):
        self._check_batch()
        return self._op(_lib.OP_CINV, vec)

    def toeplitz_gram(self, xgrids, kernel, jitter_val):
        """first row k(x0, x_j) plus nugget on c0 (`toeplitz_tensor.py:127-133`)."""
        xxs = torch.meshgrid(*xgrids, indexing="ij")
        xs = torch.stack([x.reshape(-1) for x in xxs], dim=-1)
        Krow = kernel(xs[0][None, :], xs)
        Krow[0, 0] += jitter_val
        return Krow.squeeze()

    def circulant_embed(self, Ktoe):
        """`toeplitz_tensor.py:135-143` (used only to materialise the C attribute)."""
        dims = Ktoe.shape
        for d in range(len(dims)):
            Krev = torch.flip(Ktoe, dims=(d,))
            idx = tuple([slice(None)] * d + [slice(1, -1, 1)])
            Ktoe = torch.cat([Ktoe, Krev[idx]], dim=d)
        return Ktoe

    def make_complex(self, vec):
        return torch.stack([vec, torch.zeros_like(vec)], dim=-1)

    def set_batch_shape(self, batch_shape):
        self.batch_shape = batch_shape
        self.cvec_shape = tuple(batch_shape) + self.Cc_shape

    # ---- lazily materialised spectrum attributes (toeplitz_tensor.py:20-33) ----------------
    @property
    def C(self):
        if getattr(self, "_C", None) is None:
            self._C = self.circulant_embed(self.column.view(self.dims))
        return self._C

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

    @property
    def Di_sqrt(self):
        return torch.sqrt(self.Di)
