"""G19: the reference's `svigp_fit` (`ziggy/svi_gp.py:172-442`) on config 3's OWN fit settings,
made by running the *reference* in this container with the in-memory torch-1.4 shims of
`make_golden.py` / `make_golden_grad.py` (no reference file modified, no reference source
copied; the fixture is data only).

Config 3 (`experiments-hip-gp/run_ukhousing_experiment.py`) as `experiment_util.
svigp_fit_predict_and_save` (`ziggy/misc/experiment_util.py:71-180`) sets it up:
MeanFieldToeplitzGP (fp32 model default, `hipgp.py:449-461`: noise2_init 1, no dtype passed),
Matern-3/2, sig2_init = var(y) - noise_std^2 (`run_ukhousing_experiment.py:207-208`),
ell 0.1 (`:49-50`), jitter 1e-3 (`:22`), init_Svar 0.1 (`:277`), per-observation noise std
(`uk_housing_data.py:150-168`), batch 200 (`:31`), lr 1e-2 (`:33`), schedule_lr False (`:34`,
passed through `fit_kwargs`), maxiter_cg 20 (`:71`).  The UK data are absent here: the
observations are a synthetic mean-subtracted field on the UK box with noise std .15.
N / batch = 500 as at config 3's 100k observations: the model is built with num_obs = 100,000
and `fit` sees the first 20 minibatches (4,000 observations, one epoch).

Two grids of 64 x 64 inducing points:
  * "box": over the full UK box (-5.7, 1.8) x (50, 55.5), grid spacing 0.12 / 0.087 (~ ell);
  * "fine": over a corner of the box with config 3's own 2048-point spacing (7.5 / 2047,
    5.5 / 2047), so ell / h = 27 / 37 as at 2048^2: the K conditioning and the 20-iteration
    PCG accuracy regime of the C3 grid, at a size the reference finishes on the CPU.
Recorded: the variational parameters at the start of batches STEPS (batch_callback) and
after the fit, the norms of all of them, and the per-batch ELBO trace (epoch_callback's
elbo_trace).

Result (this script's output): "box" converges (ELBO -5.28 -> -1.39 per datum over 20
batches, fp32 and fp64 alike); "fine" DIVERGES in the reference itself, fp64 included
(ELBO -4.96, -1.4e4, -5.4e8, ... -4.3e87; |theta1| x1e2-1e4 per batch; fp32 reaches inf at
batch 9 and NaN at 17): config 3's settings on its own grid spacing are unstable in the
reference's natural-gradient step, independent of the arithmetic.

fp64 also holds "{case}_alt_*": the same reference fits with NumPy's FFT in the shim (the
reference's own FFT-rounding spread, the yardstick of the GPU parity bound).

Usage:  python tests/golden/make_golden_fit_c3.py
"""
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, _np, import_reference  # noqa: E402
from make_golden_grad import _tensor_fft, _tensor_ifft  # noqa: E402

NOBS_MODEL, NFIT, BSZ, MG = 100_000, 4_000, 200, 64
NOISE_SD = .15
FIT = dict(do_cuda=False, lr=1e-2, schedule_lr=False, batch_size=BSZ, epochs=1, maxiter_cg=20,
           batch_log_interval=1)
# batches whose starting parameters are stored in full (20 = after the fit); the norms of all 21
# are stored.  "fine" diverges in the reference itself (x1e4 per batch), so only its first
# steps are kept in full
STEPS = {"box": (0, 1, 2, 5, 10, 20), "fine": (0, 1, 2, 3)}
UK_X, UK_Y = (-5.7, 1.8), (50., 55.5)
BOXES = {"box": (UK_X, UK_Y),
         "fine": ((UK_X[0], UK_X[0] + (MG - 1) * (UK_X[1] - UK_X[0]) / 2047),
                  (UK_Y[0], UK_Y[0] + (MG - 1) * (UK_Y[1] - UK_Y[0]) / 2047))}


def data(case):
    (x0, x1), (y0, y1) = BOXES[case]
    rs = np.random.RandomState(19)
    u = rs.rand(NFIT, 2)
    x = np.column_stack([x0 + (x1 - x0) * u[:, 0], y0 + (y1 - y0) * u[:, 1]])
    # a smooth field at the data's own scale (lengths of a few ell) plus noise, mean removed
    t = (x - [x0, y0]) / [x1 - x0, y1 - y0]
    f = .6 * np.sin(2.3 * np.pi * t[:, 0]) * np.cos(1.7 * np.pi * t[:, 1]) + .3 * np.cos(5.1 * t[:, 0] + 3.7 * t[:, 1])
    y = f + NOISE_SD * rs.randn(NFIT)
    y = (y - y.mean())[:, None]
    s = np.full((NFIT, 1), NOISE_SD)
    return x, y, s


def gen_case(zk, hg, dtype, case, perturb=None):
    """perturb: optional callable on the fresh model (before the fit) -- the self-perturbed
    re-runs of make_golden_fit_c3_alt.py; the recorded *_init parameters are the unperturbed ones"""
    import ziggy.svi_gp  # noqa: F401  (the reference's module, imported by ziggy.hipgp)
    torch.manual_seed(19)
    (x0, x1), (y0, y1) = BOXES[case]
    x, y, s = data(case)
    sig2 = float(y.var() - NOISE_SD ** 2)
    kern = zk.Matern(nu=1.5, dtype=dtype)
    xgrids = [torch.linspace(x0, x1, MG, dtype=dtype), torch.linspace(y0, y1, MG, dtype=dtype)]
    mod = hg.MeanFieldToeplitzGP(kern, xgrids, num_obs=NOBS_MODEL, sig2_init=sig2, ell_init=.1,
                                 init_Svar=.1, learn_kernel=False, jitter_val=1e-3, dtype=dtype)
    out = {"grid0": _np(xgrids[0]), "grid1": _np(xgrids[1]), "x": x, "y": y, "s": s,
           "sig2_init": np.array(sig2),
           "theta1_init": _np(mod.global_theta1).copy(), "theta2_init": _np(mod.global_theta2).copy()}
    if perturb is not None:
        perturb(mod)
    snaps = []

    def batch_cb(m, xb, yb, sb):
        snaps.append([_np(m.global_theta1).copy(), _np(m.global_theta2).copy()])

    traces = []

    def epoch_cb(odir, m, *args, **kw):
        traces.append(list(args[15]))          # elbo_trace (positional, svi_gp.py:405-409)
        return (None,) * 6

    with tempfile.TemporaryDirectory() as odir:
        mod.fit(odir, x, y, s, None, None, None, None, None, None,
                batch_callback=batch_cb, epoch_callback=epoch_cb, learn_kernel=False, **FIT)
    batch_cb(mod, None, None, None)
    assert len(snaps) == NFIT // BSZ + 1
    out["steps"] = np.array(STEPS[case])
    out["theta1_steps"] = np.stack([snaps[k][0] for k in STEPS[case]])
    out["theta2_steps"] = np.stack([snaps[k][1] for k in STEPS[case]])
    out["theta1_norm"] = np.array([np.linalg.norm(t[0]) for t in snaps])
    out["theta2_norm"] = np.array([np.linalg.norm(t[1]) for t in snaps])
    out["elbo_trace"] = np.array(traces[0])
    return out


def _np_fft(x, signal_ndim, normalized=False):
    dims = tuple(range(-signal_ndim, 0))
    c = torch.view_as_complex(x.contiguous()).numpy()
    return torch.view_as_real(torch.from_numpy(np.ascontiguousarray(np.fft.fftn(c, axes=dims))))


def _np_ifft(x, signal_ndim, normalized=False):
    dims = tuple(range(-signal_ndim, 0))
    c = torch.view_as_complex(x.contiguous()).numpy()
    return torch.view_as_real(torch.from_numpy(np.ascontiguousarray(np.fft.ifftn(c, axes=dims))))


def main():
    zk, tt, te, cg, hg = import_reference()
    torch.Tensor.fft = _tensor_fft
    torch.Tensor.ifft = _tensor_ifft
    torch.set_num_threads(8)
    for dtype, tag in ((torch.float64, "f64"), (torch.float32, "f32")):
        res = {}
        for case in ("box", "fine"):
            for k, v in gen_case(zk, hg, dtype, case).items():
                res[f"{case}_{k}"] = v
            print(tag, case, "elbo", res[f"{case}_elbo_trace"][[0, 1, 5, 10, -1]], flush=True)
        if dtype == torch.float64:
            # the reference's own sensitivity to FFT rounding: the same fp64 fits with the shim's
            # FFT swapped for NumPy's pocketfft (another exact C2C FFT, other rounding).  The
            # 20-iteration PCG of every natural-gradient step is unconverged, so its rounding
            # reaches the iterates at ~1e-5 ("box") and ~5e-2 ("fine", ill-conditioned) per
            # step: the GPU parity bound is 4x this spread (SURVEY §8(c) rule)
            proxy = tt.torch
            saved = (type(proxy).fft, type(proxy).ifft)
            type(proxy).fft, type(proxy).ifft = staticmethod(_np_fft), staticmethod(_np_ifft)
            try:
                for case in ("box", "fine"):
                    alt = gen_case(zk, hg, dtype, case)
                    for k in ("theta1_steps", "theta2_steps", "theta1_norm", "theta2_norm", "elbo_trace"):
                        res[f"{case}_alt_{k}"] = alt[k]
                    print(tag, case, "alt-FFT spread at step 1:",
                          np.linalg.norm(alt["theta1_steps"][1] - res[f"{case}_theta1_steps"][1]) /
                          np.linalg.norm(res[f"{case}_theta1_steps"][1]), flush=True)
            finally:
                type(proxy).fft, type(proxy).ifft = saved
        np.savez_compressed(os.path.join(OUT, f"G19_{tag}.npz"), **res)
        print("wrote", tag)


if __name__ == "__main__":
    main()
