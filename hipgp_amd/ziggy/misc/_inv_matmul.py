"""InvMatmul autograd Function (`ziggy/misc/_inv_matmul.py:9-64`).

forward: no-grad PCG solve (hgp_pcg_solve).  backward: right_grad = K^{-1} grad_output by a
second solve, as the reference does (`:27-50`).  The Toeplitz-column gradient
(`:52`, gpytorch's sym_toeplitz_derivative_quadratic_form) is SURVEY §8(f) row 4 and is
not built in this round: asking for it raises instead of returning something wrong.
"""
import torch
from torch.autograd import Function


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
        if ctx.needs_input_grad[1]:
            raise NotImplementedError("gradient w.r.t. the Toeplitz column (kernel "
                                      "hyper-parameters) is SURVEY §8(f) row 4, not built yet")
        right_grad = None
        if ctx.needs_input_grad[2]:
            right_grad = InvMatmul.apply(ctx.toeplitz_tensor, ctx.toeplitz_tensor.column,
                                         grad_output, True, ctx.maxiter, ctx.tol)
        return None, None, right_grad, None, None, None
