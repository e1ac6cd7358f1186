"""Config 3 on its own settings at full size (GPU box): the reference's fit driver
(`svigp_fit`, `svi_gp.py:172-442`, here hipgp_amd/ziggy/svi_gp.py) for 20 minibatches on a
2048 x 2048 inducing grid over the UK box (-5.7, 1.8) x (50, 55.5), MeanFieldToeplitzGP,
Matern-3/2, ell 0.1, jitter 1e-3, init_Svar 0.1, sig2 = var(y) - noise^2, batch 200, constant
lr 1e-2, maxiter_cg 20, N = 100k (num_obs; the fit sees 20 batches) -- the settings of
`run_ukhousing_experiment.py:22,31,33,49-50,207-208,277` through `experiment_util.py:71-180`.
Synthetic observations (the UK data are absent): the field of tests/golden/make_golden_fit_c3.py
on the whole box, noise std .15.

One JSON line per dtype: per-batch wall time (synchronised in the batch callback), the
500-batch epoch estimate at B = 200, the ELBO trace and |theta1| per batch.  G19 "fine" shows
the reference's own trajectory at this grid spacing diverging (tests/test_fit_c3_gpu.py).

    python tools/c3_step.py [--dtype f32,f64] [--batches 20] > gpurun_out/c3_fit.jsonl
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))


def field(x, box):
    (x0, x1), (y0, y1) = box
    t = (x - [x0, y0]) / [x1 - x0, y1 - y0]
    return .6 * np.sin(2.3 * np.pi * t[:, 0]) * np.cos(1.7 * np.pi * t[:, 1]) + .3 * np.cos(5.1 * t[:, 0] + 3.7 * t[:, 1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="f32,f64")
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--m", type=int, default=2048)
    a = ap.parse_args()
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    box = ((-5.7, 1.8), (50., 55.5))
    N, bsz, sd = 100_000, 200, .15
    nfit = a.batches * bsz
    rs = np.random.RandomState(3)
    u = rs.rand(nfit, 2)
    x = np.column_stack([box[0][0] + 7.5 * u[:, 0], box[1][0] + 5.5 * u[:, 1]])
    y = field(x, box) + sd * rs.randn(nfit)
    y = (y - y.mean())[:, None]
    s = np.full((nfit, 1), sd)
    sig2 = float(y.var() - sd ** 2)
    for tag in a.dtype.split(","):
        dt = torch.float64 if tag == "f64" else torch.float32
        npd = np.float64 if tag == "f64" else np.float32
        grids = [torch.linspace(*box[0], a.m, dtype=dt), torch.linspace(*box[1], a.m, dtype=dt)]
        mod = hg.MeanFieldToeplitzGP(zk.Matern(nu=1.5, dtype=dt), grids, num_obs=N, sig2_init=sig2, ell_init=.1,
                                     init_Svar=.1, learn_kernel=False, jitter_val=1e-3, dtype=dt)
        stamps, norms, traces = [], [], []

        def batch_cb(m, xb, yb, sb):
            torch.cuda.synchronize()
            stamps.append(time.perf_counter())
            norms.append(float(torch.linalg.norm(m.global_theta1.detach().double())))

        def epoch_cb(odir, m, *args, **kw):
            traces.append([float(v) for v in args[15]])
            return (None,) * 6

        with tempfile.TemporaryDirectory() as odir:
            mod.fit(odir, x.astype(npd), y.astype(npd), s.astype(npd), None, None, None, None, None, None,
                    batch_callback=batch_cb, epoch_callback=epoch_cb, do_cuda=True, lr=1e-2, schedule_lr=False,
                    batch_size=bsz, epochs=1, maxiter_cg=20, batch_log_interval=1, learn_kernel=False)
        torch.cuda.synchronize()
        stamps.append(time.perf_counter())
        dts = np.diff(stamps) * 1e3
        steady = float(np.median(dts[2:])) if len(dts) > 3 else float(np.median(dts))
        print(json.dumps({"what": "C3 svigp_fit on config 3's settings", "grid": [a.m, a.m], "M": a.m * a.m,
                          "batch": bsz, "num_obs": N, "batches": a.batches, "maxiter_cg": 20, "dtype": tag,
                          "lr": 1e-2, "ell": .1, "jitter": 1e-3, "init_Svar": .1, "sig2_init": round(sig2, 5),
                          "ms_per_batch_median": round(steady, 1), "ms_per_batch": [round(v, 1) for v in dts],
                          "epoch_s_500_batches": round(steady * 500 / 1e3, 1),
                          "elbo_trace": traces[0] if traces else None, "theta1_norm": norms}), flush=True)
        del mod
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
