"""compute_kn phase split of a BASELINE config (GPU box): set-up (ToeplitzTensor: the fp64
spectra), the PCG (inv_matmul) and R^T, each synchronised, median of 3.

    python tools/kn_phases.py --only C5,C4"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_configs import BOX, CONFIGS, kernel  # noqa: E402


def med(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="C5,C4")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from hipgp_amd.kuf import kuf_grid
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    for name in a.only.split(","):
        dims, (kind, nu), params, jitter, B, maxiter, tol, _ = CONFIGS[name]
        d = len(dims)
        k = kernel(kind, nu, torch.float32)
        kf = lambda x, y: k.forward(x, y, params=params)
        grids = [torch.linspace(lo, hi, m, device=dev) for (lo, hi), m in zip(BOX[d], dims)]
        g = torch.Generator(device="cpu").manual_seed(42)
        lo = torch.tensor([b[0] for b in BOX[d]])
        hi = torch.tensor([b[1] for b in BOX[d]])
        xobs = (lo + (hi - lo) * torch.rand(B, d, generator=g)).to(dev)
        Knm = kuf_grid(k, grids, xobs, params)
        out = {"config": name}
        out["setup_s"] = med(lambda: ToeplitzTensor(grids, kf, batch_shape=None, jitter_val=jitter))
        T = ToeplitzTensor(grids, kf, batch_shape=None, jitter_val=jitter)
        out["pcg_s"] = med(lambda: T.inv_matmul(Knm, do_precond=True, maxiter=maxiter, tol=tol))
        d0 = T.inv_matmul(Knm, do_precond=True, maxiter=maxiter, tol=tol)
        out["rt_s"] = med(lambda: T._matmul_by_RT(d0))
        print(json.dumps(out), flush=True)
        del T, d0, Knm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
