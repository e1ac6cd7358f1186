"""C3 minibatch step timing (GPU box): one `svigp_fit` minibatch (`svi_gp.py:172-442` via
hipgp_amd/ziggy/svi_gp.py) on the C3 shape -- 2048 x 2048 inducing grid on [-1, 1]^2, Matern-3/2
(ell 0.02, nugget 1e-2), N = 100k synthetic observations, batch 1000 (`experiment_util.py:44-50`),
PCG maxiter 20: zero grads, elbo_and_grad (fused Kuf + compute_kn + statistics), with learned
kernel the hyper backward + Adam step, the natural-gradient SGD step (lr 0.01, the svi_gp.py
default).  One JSON line per (model, learn_kernel, batch).

    python tools/c3_step.py > gpurun_out/c3_step.jsonl
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    dev = torch.device("cuda", 0)
    dt = torch.float32
    m, N, maxiter = 2048, 100_000, 20
    rng = np.random.default_rng(7)
    x = rng.uniform(-1, 1, size=(N, 2))
    y = (np.sin(3 * x[:, 0]) * np.cos(2 * x[:, 1]) + 0.1 * rng.standard_normal(N))[:, None]
    s = np.full((N, 1), 0.1)
    grids = [torch.linspace(-1, 1, m, dtype=dt)] * 2
    # (model, learned kernel, batch): the learned-kernel step keeps autograd graphs of several
    # (batch, M) tensors (16 GB each at batch 1000), so it runs at the fit default batch 256
    for cls, learn_kernel, bsz in (("MeanFieldToeplitzGP", False, 1000), ("MeanFieldToeplitzGP", True, 256)):
        mod = getattr(hg, cls)(zk.Matern(nu=1.5, dtype=dt), grids, num_obs=N, sig2_init=1., ell_init=.02,
                                jitter_val=1e-2, noise2_init=.01, learn_kernel=learn_kernel, dtype=dt).cuda_params(0)
        X = torch.tensor(x, dtype=dt, device=dev)
        Y = torch.tensor(y, dtype=dt, device=dev)
        S = torch.tensor(s, dtype=dt, device=dev)
        nat = torch.optim.SGD([mod.global_theta1, mod.global_theta2], lr=0.01)   # svi_gp.py default lr
        hyp = torch.optim.Adam([mod.log_ell, mod.log_sig2], lr=1e-3) if learn_kernel else None

        def step(b):
            sl = slice(b * bsz, (b + 1) * bsz)
            nat.zero_grad()
            if hyp is not None:
                hyp.zero_grad()
            lval = mod.elbo_and_grad(xbatch=X[sl], ybatch=Y[sl], noise_std_batch=S[sl], maxiter_cg=maxiter)
            if hyp is not None:
                (-lval).backward()
                hyp.step()
            nat.step()
            return lval

        elbos = [float(step(b)) for b in range(2)]
        torch.cuda.synchronize()
        K = 10
        t0 = time.perf_counter()
        for b in range(2, 2 + K):
            lval = step(b)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / K * 1e3
        print(json.dumps({"what": "C3 svigp_fit minibatch step", "model": cls, "learn_kernel": learn_kernel,
                          "grid": [m, m], "M": m * m, "batch": bsz, "maxiter_cg": maxiter, "dtype": "f32",
                          "ms_per_step": round(ms, 3), "epoch_s_100k": round(ms * (N // bsz) / 1e3, 3),
                          "elbo_first": elbos, "elbo_last": float(lval), "steps_timed": K}), flush=True)
        del mod, nat, hyp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
