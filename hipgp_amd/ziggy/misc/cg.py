"""Batched (P)CG with the reference recurrences (`ziggy/misc/cg.py`).

conj_grad2 (row layout, `cg.py:44-80`) and conj_grad (column layout, `cg.py:5-41`).
When the operator is a ToeplitzTensor's `_matmul_by_K` (and the preconditioner, if any, its
`_matmul_by_Cinv`), the whole loop runs as fused HIP kernels (hgp_pcg_solve /
hgp_pcg_begin+step): the early-exit test is a device flag, not a host sync per iteration.
Any other callables run the same recurrence with device row-dots from libhipgp.
"""
import torch

from hipgp_amd.plan import rowdot


class ColumnOp:
    """x (M, L) -> op(x^T)^T for a libhipgp plan: the column-layout operator lambdas that
    `gram_solve` hands `conj_grad` (`toeplitz_expanded.py:46-49`), as an object `conj_grad`
    recognises, so that the whole column-layout solve runs as hgp_pcg_solve(LAYOUT_COLS)."""

    def __init__(self, plan, op):
        self.plan, self.op = plan, op

    def __call__(self, x):
        return self.plan.apply(self.op, x.t().contiguous()).t()


def _cols_fastpath(A_mul, precond):
    from hipgp_amd import _lib
    if not isinstance(A_mul, ColumnOp) or A_mul.op != _lib.OP_K:
        return None
    if precond is None:
        return A_mul.plan, False
    if isinstance(precond, ColumnOp) and precond.plan is A_mul.plan and precond.op == _lib.OP_CINV:
        return A_mul.plan, True
    return None


def _toeplitz_fastpath(A_mul, precond):
    owner = getattr(A_mul, "__self__", None)
    fn = getattr(A_mul, "__func__", None)
    if owner is None or fn is None or fn.__name__ != "_matmul_by_K" or not hasattr(owner, "_plan"):
        return None
    if precond is None:
        return owner, False
    if getattr(precond, "__self__", None) is owner and getattr(precond, "__func__", None) is not None \
            and precond.__func__.__name__ == "_matmul_by_Cinv":
        return owner, True
    return None


def _generic(A_mul, b, precond, maxiter, tol, callback):
    """cg.py:44-80 with arbitrary callables; dots by hgp_rowdot (device)."""
    if precond is None:
        precond = lambda x: x
    x = torch.zeros_like(b)
    r = b - A_mul(x)
    z = precond(r)
    p = z
    for n in range(maxiter):
        rs = rowdot(r, z)
        Ap = A_mul(p)
        alpha = rs / rowdot(p, Ap)
        x = x + alpha.unsqueeze(-1) * p
        r = r - alpha.unsqueeze(-1) * Ap
        rnew = rowdot(r, r)
        if torch.all(torch.sqrt(rnew) < tol):
            break
        z = precond(r)
        beta = rowdot(z, r) / rs
        p = z + beta.unsqueeze(-1) * p
        if callback is not None:
            callback(n, x)
    return x


def conj_grad2(A_mul, b, precond=None, maxiter=20, tol=1e-10, callback=None):
    """A^{-1} b for b (bsz, M); per-RHS alpha/beta; stops when ALL sqrt(r.r) < tol."""
    fp = _toeplitz_fastpath(A_mul, precond)
    if fp is not None:
        owner, use_p = fp
        if callback is None:
            return owner._plan.pcg(b, maxiter, tol, precond=use_p)
        return owner._plan.pcg_steps(b, maxiter, tol, precond=use_p, callback=callback)
    return _generic(A_mul, b, precond, maxiter, tol, callback)


def conj_grad(A_mul, b, precond=None, maxiter=20, tol=1e-10, callback=None):
    """Column layout: b (M, L), dim=0 dots (`cg.py:5-41`); same recurrence per column.
    ColumnOp operators of one plan (K, and C^-1 as the preconditioner) run as one fused
    hgp_pcg_solve in LAYOUT_COLS; any other callables run the generic recurrence."""
    from hipgp_amd import _lib
    fp = _cols_fastpath(A_mul, precond)
    if fp is not None:
        plan, use_p = fp
        if callback is None:
            return plan.pcg(b, maxiter, tol, precond=use_p, layout=_lib.LAYOUT_COLS)
        return plan.pcg_steps(b, maxiter, tol, precond=use_p, callback=callback, layout=_lib.LAYOUT_COLS)
    At = lambda y: A_mul(y.t()).t()
    Pt = None if precond is None else (lambda y: precond(y.t()).t())
    cb = None if callback is None else (lambda n, x: callback(n, x.t()))
    return conj_grad2(At, b.t().contiguous(), precond=Pt, maxiter=maxiter, tol=tol, callback=cb).t()
