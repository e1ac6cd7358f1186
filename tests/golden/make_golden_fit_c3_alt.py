"""G19 "fine": nine self-perturbed re-runs of the *reference*'s fp64 `svigp_fit` on config 3's
own grid spacing (`make_golden_fit_c3.py`'s "fine" case), as `make_golden_clamp_alt.py` does for
the clamped solves.  G19 itself holds ONE alternative run (NumPy's FFT in the shim); one sample
of a chaotic spread is a thin yardstick, so this fixture holds nine:

* alt0: NumPy's pocketfft in place of the shim's torch FFT (the existing G19 "fine_alt" run);
* alt1..alt4: the reference's own FFT, every Toeplitz column the fit builds (`ToeplitzTensor.
  toeplitz_gram`, one per minibatch) moved by one unit in the last place per element (four
  seeds) -- the same problem at fp64 rounding, another rounding path through every solve (the
  variational parameters would not do: k_n does not depend on them, so the natural-gradient
  step, affine in them, carries their last-place moves along unamplified);
* alt5..alt8: every FFT output perturbed at the rounding level of an fp FFT of another
  algorithm or length (eps * max|X| * sqrt(log2 N) * N(0, 1), four seeds) -- what a different
  transform (the L-grid route of the GPU path) does to the same arithmetic.

Recorded per run: its difference from the reference's own run (G19 "fine") in the variational
parameters at the start of batches STEPS["fine"], in fp32 (the bound reads distances of ~1e-2).
The GPU parity bound (`tests/test_fit_c3_gpu.py`) is 10x the largest of the nine distances from
the reference's own trajectory.  Test infrastructure only: same in-memory shims as
`make_golden.py` (no reference file modified, no reference source copied; the fixture is data).

Usage:  python tests/golden/make_golden_fit_c3_alt.py      (writes tests/golden/G19_fine_alt.npz)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, import_reference  # noqa: E402
from make_golden_clamp_alt import _noisy, _ulp  # noqa: E402
from make_golden_fit_c3 import _np_fft, _np_ifft, gen_case  # noqa: E402
from make_golden_grad import _tensor_fft, _tensor_ifft  # noqa: E402


def main():
    zk, tt, te, cg, hg = import_reference()
    torch.Tensor.fft = _tensor_fft
    torch.Tensor.ifft = _tensor_ifft
    torch.set_num_threads(8)
    ref = np.load(os.path.join(OUT, "G19_f64.npz"))
    proxy = tt.torch
    torch_fft = (type(proxy).__dict__["fft"], type(proxy).__dict__["ifft"])
    path = os.path.join(OUT, "G19_fine_alt.npz")
    # resumable: runs already in the fixture are kept (each run takes minutes on 8 CPU threads)
    res = dict(np.load(path)) if os.path.exists(path) else {}
    for k in list(res):          # the older format kept the parameters themselves
        if k.endswith("_steps") and k.startswith("alt"):
            res[k.replace("_steps", "_diff")] = (res.pop(k) - ref["fine_" + k.split("_", 1)[1]]).astype(np.float32)
    gram = tt.ToeplitzTensor.toeplitz_gram       # the reference's method (in-memory wrap only)
    for a in range(9):
        if f"alt{a}_theta1_diff" in res:
            continue
        if a == 0:
            type(proxy).fft, type(proxy).ifft = staticmethod(_np_fft), staticmethod(_np_ifft)
        elif a <= 4:
            calls = [0]

            def gram_ulp(self, xgrids, kernel, jitter_val, a=a, calls=calls):
                calls[0] += 1
                return _ulp(gram(self, xgrids, kernel, jitter_val), 1000 * a + calls[0])
            tt.ToeplitzTensor.toeplitz_gram = gram_ulp
        else:
            f0, i0 = torch_fft[0].__func__, torch_fft[1].__func__
            type(proxy).fft, type(proxy).ifft = staticmethod(_noisy(f0, 10 * a)), staticmethod(_noisy(i0, 10 * a + 1))
        try:
            out = gen_case(zk, hg, torch.float64, "fine")
        finally:
            type(proxy).fft, type(proxy).ifft = torch_fft
            tt.ToeplitzTensor.toeplitz_gram = gram
        assert np.array_equal(out["theta1_init"], ref["fine_theta1_init"]), "initial state differs from G19"
        for name in ("theta1", "theta2"):
            res[f"alt{a}_{name}_diff"] = (out[f"{name}_steps"] - ref[f"fine_{name}_steps"]).astype(np.float32)
        for j in range(1, len(out["steps"])):
            s = np.linalg.norm(out["theta1_steps"][j] - ref["fine_theta1_steps"][j]) / np.linalg.norm(ref["fine_theta1_steps"][j])
            print(f"alt{a} step {out['steps'][j]}: theta1 spread {s:.3e}", flush=True)
        res["steps"] = out["steps"]
        np.savez_compressed(path, **res)
    print("wrote G19_fine_alt.npz")


if __name__ == "__main__":
    main()
