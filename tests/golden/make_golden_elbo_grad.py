"""Golden vectors for kernel/noise hyper-parameter learning through `elbo_and_grad` (the
reference's fit loop calls `(-lval).backward()` when learn_kernel / learn_noise is set,
`svi_gp.py:317-326`), made by running the *reference* in this container with the same
in-memory torch-1.4 shims as `make_golden.py` / `make_golden_grad.py` (no reference file
modified, no reference source copied; the fixtures are data only).

G16 (mean-field) / G17 (block, 2x3 blocks of the expanded grid), fp64 and fp32:
  MeanFieldToeplitzGP / BlockToeplitzGP on a 12x10 grid, Matern-3/2, learn_kernel=True,
  learn_noise=True, 40 point observations, maxiter_cg=20, random variational parameters.
  Recorded: the ELBO, theta1/theta2 grads (natural gradient, `hipgp.py:194-276`) and, after
  `elbo.backward()`, the grads of log_sig2, log_ell, log_noise2 (`_inv_matmul.py:27-64`,
  `gpt_toeplitz.py:169-209`, autograd of `toeplitz_tensor.py:20-31,85-97`).

Usage:  python tests/golden/make_golden_elbo_grad.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, _np, import_reference  # noqa: E402
from make_golden_grad import _tensor_fft, _tensor_ifft  # noqa: E402


def gen_case(zk, hg, dtype, tag, name, family):
    torch.manual_seed(16)
    rs = np.random.RandomState(16)
    kern = zk.Matern(nu=1.5, dtype=dtype)
    xgrids = [torch.linspace(-1, 1, 12, dtype=dtype), torch.linspace(-1, 1, 10, dtype=dtype)]
    kw = dict(sig2_init=1.2, ell_init=.3, noise2_init=.05, learn_kernel=True, learn_noise=True, dtype=dtype)
    if family == "mean-field":
        mod = hg.MeanFieldToeplitzGP(kern, xgrids, num_obs=400, **kw)
    else:
        mod = hg.BlockToeplitzGP(kern, xgrids, num_obs=400, block_sizes=[2, 3], **kw)
    Mp = mod.Mprime
    with torch.no_grad():
        mod.global_theta1.copy_(torch.tensor(rs.randn(Mp, 1) * .3, dtype=dtype))
        if family == "mean-field":
            mod.global_theta2.copy_(torch.tensor(-.5 / (.05 + rs.rand(Mp, 1)), dtype=dtype))
        else:
            nb, bs, _ = mod.global_theta2.shape
            A = rs.randn(nb, bs, bs) * .2
            S = A @ A.transpose(0, 2, 1) + .1 * np.eye(bs)[None]
            mod.global_theta2.copy_(torch.tensor(-.5 * np.linalg.inv(S), dtype=dtype))
    xobs = torch.tensor(rs.rand(40, 2) * 1.8 - .9, dtype=dtype)
    yobs = torch.tensor(rs.randn(40, 1), dtype=dtype)
    elbo = mod.elbo_and_grad(xobs, yobs, maxiter_cg=20)
    out = {"grid0": _np(xgrids[0]), "grid1": _np(xgrids[1]), "xobs": _np(xobs), "yobs": _np(yobs),
           "theta1": _np(mod.global_theta1), "theta2": _np(mod.global_theta2),
           "elbo": np.array(float(elbo)), "theta1_grad": _np(mod.global_theta1.grad),
           "theta2_grad": _np(mod.global_theta2.grad)}
    elbo.backward()
    out.update({"log_sig2_grad": np.array(float(mod.log_sig2.grad)),
                "log_ell_grad": np.array(float(mod.log_ell.grad)),
                "log_noise2_grad": np.array(float(mod.log_noise2.grad))})
    np.savez_compressed(os.path.join(OUT, f"{name}_{tag}.npz"), **out)


def main():
    zk, tt, te, cg, hg = import_reference()
    torch.Tensor.fft = _tensor_fft
    torch.Tensor.ifft = _tensor_ifft
    torch.set_num_threads(8)
    for dtype, tag in ((torch.float64, "f64"), (torch.float32, "f32")):
        gen_case(zk, hg, dtype, tag, "G16", "mean-field")
        gen_case(zk, hg, dtype, tag, "G17", "block")
        print("wrote", tag)


if __name__ == "__main__":
    main()
