"""Alt-FFT fixtures for the clamped 20-iteration goldens (G4a-c, G7): the *reference*'s
`_solve(maxiter=20, precond)` and its compute_kn-equivalent `R^T K^-1 v` (the keys
`solve_p1_it20` / `kn_it20` of `make_golden.py`'s `_grid_case`), re-run with the shim's FFT
swapped for NumPy's pocketfft -- another exact C2C FFT with other rounding.

Why: at the 1e-6 spectrum clamp 20 PCG iterations amplify rounding chaotically, so the
reference disagrees with ITSELF under a different FFT by far more than the ops' rounding.  That
self-spread is the yardstick the parity tests hold these cases to (the SURVEY §8(c) rule:
within 4x the reference's own implementation spread), next to the true-residual check.  One
alternative run is one sample of a chaotic spread, so the fixture holds nine: NumPy's FFT
("alt0"), the reference's own torch FFT on the right-hand sides perturbed by one unit in the
last place of every element (four seeds, "alt1".."alt4"), and the reference with every FFT
output perturbed at the rounding level of an fp FFT of another algorithm or length
("alt5".."alt8": each element + eps * max|X| * sqrt(log2 N) * N(0, 1), four seeds).  NumPy's and
torch's CPU FFTs are both pocketfft, so alt0..alt4 share the reference's rounding pattern; an
implementation with other transform lengths (the L-grid route here) does not, and at the clamp
(1/D up to 1e6) those rounding differences are what 20 iterations amplify -- alt5..alt8 model
them.  The yardstick is the largest of the nine.

Test infrastructure only (same shims as `make_golden.py`: no reference file modified, no
reference source copied; the fixture is data only).

Usage:  python tests/golden/make_golden_clamp_alt.py     (writes tests/golden/G4a_alt.npz, ...)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, _np, import_reference  # noqa: E402
from make_golden_fit_c3 import _np_fft, _np_ifft  # noqa: E402

# name: (dims, lo, hi, kernel (kind, nu), params, jitter, B) -- as make_golden.main()
CASES = {
    "G4a": ((32, 24), (-1, -1), (1, 1), ("sqexp", None), (1., .5), 1e-3, 3),
    "G4b": ((32, 24), (-1, -1), (1, 1), ("matern", .5), (1., 5.), 1e-3, 3),
    "G4c": ((32, 24), (-1, -1), (1, 1), ("matern", 2.5), (1., 1.), 1e-3, 3),
    "G7": ((37, 3), (-1, 0), (1, .5), ("matern", 1.5), (1., .4), 1e-3, 5),
}


def _noisy(fft, seed):
    """an FFT whose outputs carry independent rounding-level noise (another algorithm's rounding)"""
    gen = torch.Generator().manual_seed(seed)

    def f(x, signal_ndim, normalized=False):
        y = fft(x, signal_ndim)
        n = int(np.prod(x.shape[-1 - signal_ndim:-1]))
        eps = float(torch.finfo(y.dtype).eps) / 2
        amp = eps * float(y.abs().max()) * float(np.sqrt(max(1.0, np.log2(n))))
        return y + amp * torch.randn(y.shape, generator=gen, dtype=torch.float64).to(y.dtype)
    return f


def _ulp(t, seed):
    """t moved by one unit in the last place, up or down per element (seeded)"""
    gs = torch.Generator().manual_seed(seed)
    sgn = torch.randint(0, 2, t.shape, generator=gs).bool()
    return torch.where(sgn, torch.nextafter(t, torch.full_like(t, np.inf)),
                       torch.nextafter(t, torch.full_like(t, -np.inf)))


def run(zk, tt, dtype, name, ulp_seed=None):
    dims, lo, hi, (kind, nu), params, jitter, B = CASES[name]
    kern = zk.SqExp(dtype=dtype) if kind == "sqexp" else zk.Matern(nu=nu, dtype=dtype)
    kfun = lambda x, y: kern.forward(x, y, params=params)
    xgrids = [torch.linspace(lo[d], hi[d], dims[d], dtype=dtype) for d in range(len(dims))]
    T = tt.ToeplitzTensor(xgrids, kfun, batch_shape=None, jitter_val=jitter)
    M = int(np.prod(dims))
    g = torch.Generator().manual_seed(0)
    v = torch.randn(B, M, generator=g, dtype=torch.float64).to(dtype)
    v0 = v.clone()
    if ulp_seed is not None:      # +-1 ulp on every element: another rounding path, same problem
        v = _ulp(v, ulp_seed)
    T.set_batch_shape((B,))
    return {"v": _np(v0),
            "solve_p1_it20": _np(T._solve(v, do_precond=True, maxiter=20, tol=1e-8)),
            "kn_it20": _np(T._matmul_by_RT(T.inv_matmul(v, do_precond=True, maxiter=20, tol=1e-8)))}


def main():
    zk, tt, te, cg, hg = import_reference()
    torch.set_num_threads(8)
    proxy = tt.torch
    torch_fft = (type(proxy).__dict__["fft"], type(proxy).__dict__["ifft"])   # the staticmethod objects
    for name in CASES:
        res = {}
        for dtype, tag in ((torch.float64, "f64"), (torch.float32, "f32")):
            ref = np.load(os.path.join(OUT, f"{name}_{tag}.npz"))
            for a in range(9):
                if a == 0:
                    type(proxy).fft, type(proxy).ifft = staticmethod(_np_fft), staticmethod(_np_ifft)
                    out = run(zk, tt, dtype, name)
                    type(proxy).fft, type(proxy).ifft = torch_fft
                elif a <= 4:
                    out = run(zk, tt, dtype, name, ulp_seed=a)
                else:
                    f0, i0 = torch_fft[0].__func__, torch_fft[1].__func__
                    type(proxy).fft, type(proxy).ifft = staticmethod(_noisy(f0, 10 * a)), staticmethod(_noisy(i0, 10 * a + 1))
                    out = run(zk, tt, dtype, name)
                    type(proxy).fft, type(proxy).ifft = torch_fft
                assert np.array_equal(out["v"], ref["v"]), (name, tag, "inputs differ from the golden")
                for k in ("solve_p1_it20", "kn_it20"):
                    res[f"{tag}_{k}_alt{a}"] = out[k]
                    spread = np.linalg.norm(out[k] - ref[k]) / np.linalg.norm(ref[k])
                    print(name, tag, k, f"alt{a} spread", f"{spread:.3e}", flush=True)
        np.savez_compressed(os.path.join(OUT, f"{name}_alt.npz"), **res)


if __name__ == "__main__":
    main()
