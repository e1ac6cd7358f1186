"""Golden trajectories of the reference's minibatch natural-gradient driver `svigp_fit`
(`ziggy/svi_gp.py:172-442`, reached through `SviGP.fit`, `:99-114`), made by running the
*reference* in this container with the in-memory torch-1.4 shims of `make_golden.py` /
`make_golden_grad.py` (no reference file modified, no reference source copied; the fixture
is data only).

G18 (fp64 and fp32): MeanFieldToeplitzGP on a 20 x 20 grid over [-1, 1]^2, Matern-3/2
(sig2 1, ell .15), 64 point observations with per-observation noise sd .1, one epoch of
4 minibatches of 16, maxiter_cg 20, SGD lr .05 with StepLR decay .9 per batch:
  * case "ng": natural gradient only;
  * case "hk": learn_kernel=True (Adam on log_ell, log_sig2, kernel_lr .05).
Recorded: the initial variational parameters, the parameters at the start of every batch
(batch_callback) and after the fit, and the ELBO trace (epoch_callback's elbo_trace).

Usage:  python tests/golden/make_golden_fit.py
"""
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, _np, import_reference  # noqa: E402
from make_golden_grad import _tensor_fft, _tensor_ifft  # noqa: E402

FIT = dict(do_cuda=False, lr=.05, step_decay=.9, batch_size=16, epochs=1, maxiter_cg=20,
           kernel_lr=.05, batch_log_interval=1)


def gen_case(zk, hg, dtype, case):
    import ziggy.svi_gp  # noqa: F401  (the reference's module, imported by ziggy.hipgp)
    torch.manual_seed(18)
    rs = np.random.RandomState(18)
    kern = zk.Matern(nu=1.5, dtype=dtype)
    xgrids = [torch.linspace(-1, 1, 20, dtype=dtype), torch.linspace(-1, 1, 20, dtype=dtype)]
    learn = case == "hk"
    mod = hg.MeanFieldToeplitzGP(kern, xgrids, num_obs=64, sig2_init=1., ell_init=.15, noise2_init=.01,
                                 init_Svar=.5, learn_kernel=learn, learn_noise=False, dtype=dtype)
    x = rs.rand(64, 2) * 1.8 - .9
    y = np.sin(3 * x[:, :1]) * np.cos(2 * x[:, 1:]) + .1 * rs.randn(64, 1)
    s = np.full((64, 1), .1)
    out = {"grid0": _np(xgrids[0]), "grid1": _np(xgrids[1]), "x": x, "y": y, "s": s,
           # copies: _np views the parameter's storage, which the fit updates in place
           "theta1_init": _np(mod.global_theta1).copy(), "theta2_init": _np(mod.global_theta2).copy()}
    snaps = []

    def batch_cb(m, xb, yb, sb):
        snaps.append([_np(m.global_theta1).copy(), _np(m.global_theta2).copy(),
                      float(m.log_sig2), float(m.log_ell)])

    traces = []

    def epoch_cb(odir, m, *args, **kw):
        traces.append(list(args[15]))          # elbo_trace (positional, svi_gp.py:405-409)
        return (None,) * 6

    with tempfile.TemporaryDirectory() as odir:
        mod.fit(odir, x, y, s, None, None, None, None, None, None,
                batch_callback=batch_cb, epoch_callback=epoch_cb, learn_kernel=learn, **FIT)
    batch_cb(mod, None, None, None)
    out["theta1_steps"] = np.stack([t[0] for t in snaps])
    out["theta2_steps"] = np.stack([t[1] for t in snaps])
    out["log_sig2_steps"] = np.array([t[2] for t in snaps])
    out["log_ell_steps"] = np.array([t[3] for t in snaps])
    out["elbo_trace"] = np.array(traces[0])
    return out


def main():
    zk, tt, te, cg, hg = import_reference()
    torch.Tensor.fft = _tensor_fft
    torch.Tensor.ifft = _tensor_ifft
    torch.set_num_threads(8)
    for dtype, tag in ((torch.float64, "f64"), (torch.float32, "f32")):
        res = {}
        for case in ("ng", "hk"):
            for k, v in gen_case(zk, hg, dtype, case).items():
                res[f"{case}_{k}"] = v
        np.savez_compressed(os.path.join(OUT, f"G18_{tag}.npz"), **res)
        print("wrote", tag, {k: v.shape for k, v in res.items() if k.endswith("steps")})


if __name__ == "__main__":
    main()
