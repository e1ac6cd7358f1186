"""Set-up (ToeplitzTensor construction: fp64 spectra) of a BASELINE config, repeated, for
rocprofv3 --kernel-trace --stats (GPU box).   python tools/setup_prof.py --cfg C5"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_configs import BOX, CONFIGS, kernel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="C5")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    dims, (kind, nu), params, jitter, B, maxiter, tol, _ = CONFIGS[a.cfg]
    k = kernel(kind, nu, torch.float32)
    kf = lambda x, y: k.forward(x, y, params=params)
    grids = [torch.linspace(lo, hi, m, device=dev) for (lo, hi), m in zip(BOX[len(dims)], dims)]
    for _ in range(a.reps):
        ToeplitzTensor(grids, kf, batch_shape=None, jitter_val=jitter)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
