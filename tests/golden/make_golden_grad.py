"""Golden vectors for the backward pass through the solve and the whitening,
made by running the *reference* in this container (same in-memory torch-1.4 shim as
`make_golden.py`, plus the torch-1.4 `Tensor.fft/ifft` methods `ziggy/misc/gpt_fft.py:6-14` calls;
no reference file modified, no reference source copied; the fixtures are data only).

Per case (G13: 1-D m=40; G14: 2-D 9x7; G15: 3-D 5x4x3), fp64 and fp32:
  * InvMatmul.backward (`_inv_matmul.py:27-64`): column gradient (gpytorch's
    sym_toeplitz_derivative_quadratic_form on the flattened column, `gpt_toeplitz.py:169-209`)
    and right-hand-side gradient for a random grad_output;
  * the whitening R^T (`toeplitz_tensor.py:85-97`) differentiated w.r.t. the column through
    D_sqrt = sqrt(clamp(Re FFT(embed(column)), 1e-6)) (`:20-31`);
  * K, C^-1 and R differentiated w.r.t. the column through D, 1/D, D_sqrt (`:70-83, 99-125`);
  * end to end (ziggy whitening with learn_kernel): d/d(sig2, ell) of sum(W * R^T K^{-1} Knm^T)
    with Knm and the Toeplitz column from the same kernel parameters (`hipgp.py:117-146`).

Usage:  python tests/golden/make_golden_grad.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, _np, import_reference  # noqa: E402


def _tensor_fft(self, signal_ndim, normalized=False):
    dims = tuple(range(-signal_ndim, 0))
    return torch.view_as_real(torch.fft.fftn(torch.complex(self[..., 0], self[..., 1]), dim=dims))


def _tensor_ifft(self, signal_ndim, normalized=False):
    dims = tuple(range(-signal_ndim, 0))
    return torch.view_as_real(torch.fft.ifftn(torch.complex(self[..., 0], self[..., 1]), dim=dims))


def gen_case(zk, tt, dtype, tag, name, dims, kern, params, B, seed):
    rs = np.random.RandomState(seed)
    grids = [torch.linspace(-1, 1, m, dtype=dtype) for m in dims]
    M = int(np.prod(dims))
    Mp = int(np.prod([2 * m - 2 if m > 1 else m for m in dims]))
    sig2 = torch.tensor(params[0], dtype=dtype, requires_grad=True)
    ell = torch.tensor(params[1], dtype=dtype, requires_grad=True)
    kfun = lambda x, y: kern(x, y, params=(sig2, ell))
    out = {f"grid{i}": _np(g) for i, g in enumerate(grids)}
    out["dims"] = np.array(dims)
    out["params"] = np.array(params)
    # (1) InvMatmul backward w.r.t. the column and the right-hand side
    T = tt.ToeplitzTensor(grids, kfun, batch_shape=None, jitter_val=1e-3)
    col = T.column.detach().clone().requires_grad_(True)
    R = torch.tensor(rs.randn(B, M), dtype=dtype, requires_grad=True)
    gout = torch.tensor(rs.randn(B, M), dtype=dtype)
    from ziggy.misc._inv_matmul import InvMatmul
    sol = InvMatmul.apply(T, col, R, True, 30, 1e-10)
    sol.backward(gout)
    out.update({"column": _np(T.column), "R": _np(R), "grad_out": _np(gout), "solves": _np(sol),
                "inv_column_grad": _np(col.grad), "inv_right_grad": _np(R.grad)})
    # (2) R^T differentiated w.r.t. the column through D_sqrt
    T2 = tt.ToeplitzTensor(grids, kfun, batch_shape=None, jitter_val=1e-3)
    T2.set_batch_shape((B,))
    v = torch.tensor(rs.randn(B, M), dtype=dtype)
    g = torch.tensor(rs.randn(B, Mp), dtype=dtype)
    y = T2._matmul_by_RT(v)
    (gc,) = torch.autograd.grad((y * g).sum(), T2.column)
    out.update({"rt_v": _np(v), "rt_g": _np(g), "rt_y": _np(y), "rt_column_grad": _np(gc)})
    # (3) end to end: compute_kn with learn_kernel (ziggy whitening)
    x = torch.tensor(rs.rand(B, len(dims)) * 1.6 - .8, dtype=dtype)
    mesh = torch.meshgrid(*grids, indexing="ij")
    xinduce = torch.stack([m_.reshape(-1) for m_ in mesh], dim=-1)
    Knm = kfun(x, xinduce)
    T3 = tt.ToeplitzTensor(grids, kfun, batch_shape=None, jitter_val=1e-3)
    d0 = T3.inv_matmul(Knm, do_precond=True, maxiter=30, tol=1e-10)
    kn = T3._matmul_by_RT(d0)
    W = torch.tensor(rs.randn(B, Mp), dtype=dtype)
    loss = (kn * W).sum()
    gs, ge = torch.autograd.grad(loss, (sig2, ell))
    out.update({"x": _np(x), "W": _np(W), "kn": _np(kn), "loss": np.array(float(loss)),
                "dsig2": np.array(float(gs)), "dell": np.array(float(ge))})
    # (4) the other operators differentiated w.r.t. the column through D / 1/D / D_sqrt
    #     (`toeplitz_tensor.py:70-83, 99-125`); drawn last so (1)-(3) keep their values
    T4 = tt.ToeplitzTensor(grids, kfun, batch_shape=None, jitter_val=1e-3)
    T4.set_batch_shape((B,))
    for key, fn, nin, nout in (("K", T4._matmul_by_K, M, M), ("Cinv", T4._matmul_by_Cinv, M, M),
                               ("R", T4._matmul_by_R, Mp, M)):
        xv = torch.tensor(rs.randn(B, nin), dtype=dtype)
        gv = torch.tensor(rs.randn(B, nout), dtype=dtype)
        (gc,) = torch.autograd.grad((fn(xv) * gv).sum(), T4.column, retain_graph=True)
        out.update({f"{key}_x": _np(xv), f"{key}_g": _np(gv), f"{key}_column_grad": _np(gc)})
    np.savez_compressed(os.path.join(OUT, f"{name}_{tag}.npz"), **out)


def main():
    zk, tt, te, cg, hg = import_reference()
    torch.Tensor.fft = _tensor_fft
    torch.Tensor.ifft = _tensor_ifft
    torch.set_num_threads(8)
    for dtype, tag in ((torch.float64, "f64"), (torch.float32, "f32")):
        gen_case(zk, tt, dtype, tag, "G13", (40,), zk.Matern(nu=2.5, dtype=dtype), (1., .3), 3, 13)
        gen_case(zk, tt, dtype, tag, "G14", (9, 7), zk.SqExp(dtype=dtype), (1., .4), 4, 14)
        gen_case(zk, tt, dtype, tag, "G15", (5, 4, 3), zk.Matern(nu=1.5, dtype=dtype), (1., .6), 2, 15)
        print("wrote", tag)


if __name__ == "__main__":
    main()
