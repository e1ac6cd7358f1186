"""InvMatmul autograd Function (`ziggy/misc/_inv_matmul.py:9-64`).

forward: no-grad PCG solve (hgp_pcg_solve).  backward (`:27-64`): left solves
L = K^{-1} grad_output by a second solve (always preconditioned, as the reference); the
right-hand-side gradient is L; the Toeplitz-column gradient is gpytorch's
sym_toeplitz_derivative_quadratic_form([L; R]^T, -0.5 [R; L]^T) over the flattened column
(`:52-60`), summed to the column's shape (`:62-63`).  The quadratic form runs through the
grid's factorisation (hgp_plan_dqf: the flattened-index correlation is a fold of the d-D one,
one fp64 FFT per vector pair) -- the reference's 1-D rule, evaluated in O(M log M).
"""
import torch
from torch.autograd import Function

from hipgp_amd.plan import sym_toeplitz_dqf


class InvMatmul(Function):
    @staticmethod
    def forward(ctx, toeplitz_tensor, column, right_tensor, do_precond, maxiter, tol):
        assert right_tensor.ndimension() == 2, right_tensor.ndimension()
        ctx.toeplitz_tensor = toeplitz_tensor
        with torch.no_grad():
            solves = toeplitz_tensor._solve(right_tensor, do_precond=do_precond, maxiter=maxiter,
                                            tol=tol, callback=None)
        ctx.save_for_backward(solves)
        ctx.maxiter = int(maxiter)
        ctx.tol = float(tol)
        return solves

    @staticmethod
    def backward(ctx, grad_output):
        (right_solves,) = ctx.saved_tensors
        left_solves = None
        if any(ctx.needs_input_grad):
            left_solves = InvMatmul.apply(ctx.toeplitz_tensor, ctx.toeplitz_tensor.column,
                                          grad_output, True, ctx.maxiter, ctx.tol)
        column_grad = None
        if ctx.needs_input_grad[1]:
            with torch.no_grad():
                left_vecs = torch.cat([left_solves, right_solves], 0)
                right_vecs = torch.cat([right_solves, left_solves], 0).mul(-0.5)
                plan = getattr(ctx.toeplitz_tensor, "_plan", None)
                if plan is not None:
                    column_grad = plan.dqf(left_vecs, right_vecs)
                else:
                    column_grad = sym_toeplitz_dqf(left_vecs.t(), right_vecs.t())
            column = ctx.toeplitz_tensor.column
            if column_grad.dim() > column.dim():
                column_grad = column_grad.view(-1, *column.shape).sum(0)
            column_grad = column_grad.view(column.shape)
        right_grad = left_solves if ctx.needs_input_grad[2] else None
        return None, column_grad, right_grad, None, None, None
