"""Diagnostic: where does the fp64 raw-buffer (HGP_BUF_F64) column pass go wrong?

K v on thin 2-D grids in fp64 against the fp64 oracle; prints the error map summarised over
(RHS, axis-0 index, axis-1 index) and run-to-run differences, for several RHS counts."""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ziggy_oracle as zo
from hipgp_amd import _lib
from hipgp_amd.plan import ToeplitzPlan

for s in sys.argv[1:]:
    dims = tuple(int(v) for v in s.split("x"))
    grids = [np.linspace(-1, 1, m) for m in dims]
    col = zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., .1), nu=1.5), 0.1)
    T = zo.ToeplitzOracle(col, dims)
    for B in (1, 2, 4):
        v = np.random.RandomState(0).randn(B, T.M)
        ref = T.matmul_K(v)
        P = ToeplitzPlan(dims, torch.float64, "cuda")
        P.set_column(torch.tensor(col, device="cuda"))
        vt = torch.tensor(v, device="cuda")
        ys = [P.apply(_lib.OP_K, vt).cpu().numpy() for _ in range(4)]
        err = np.abs(ys[0] - ref).reshape((B,) + dims) / np.abs(ref).max()
        bad = np.argwhere(err > 1e-12)
        rep = [float(np.abs(y - ys[0]).max()) for y in ys[1:]]
        print(dims, "B", B, "max err", f"{err.max():.2e}", "bad", len(bad), "of", err.size,
              "repeat", [f"{r:.1e}" for r in rep], flush=True)
        if len(bad):
            for ax in range(bad.shape[1]):
                u = np.unique(bad[:, ax])
                print("   axis", ax, "bad idx count", len(u), "first", u[:12].tolist(), "last", u[-6:].tolist(), flush=True)
            # error spread along axis 1 (the axis-0 line = one compact column of axis 1)
            print("   err by axis-1 index:", [f"{e:.1e}" for e in err.max(axis=(0, 1))], flush=True)
