"""Diagnostic: fp64 K and R^T of 2-D grids against the oracle (one RHS), per axis length,
plus the plan's clamped spectrum D against the oracle's."""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ziggy_oracle as zo
from hipgp_amd import _lib
from hipgp_amd.plan import ToeplitzPlan

ms = [int(v) for v in sys.argv[1].split(",")]
for m0 in ms:
    for m1 in ms:
        dims = (m0, m1)
        grids = [np.linspace(-1, 1, m) for m in dims]
        col = zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., .1), nu=1.5), 0.1)
        T = zo.ToeplitzOracle(col, dims)
        rs = np.random.RandomState(0)
        v = rs.randn(1, T.M)
        P = ToeplitzPlan(dims, torch.float64, "cuda")
        P.set_column(torch.tensor(col, device="cuda"))
        D = P.spectrum(_lib.SPEC_D).cpu().numpy()
        eD = float(np.max(np.abs(D - T.D)) / np.max(np.abs(T.D)))
        out = {"D": eD}
        for name, op, ref in (("K", _lib.OP_K, T.matmul_K(v)), ("RT", _lib.OP_RT, T.matmul_RT(v))):
            y = P.apply(op, torch.tensor(v, device="cuda")).cpu().numpy()
            out[name] = float(np.max(np.abs(y - ref)) / np.max(np.abs(ref)))
        print(dims, "H_K", [L // 2 for L in P.L_K[:2]], "H_R", [L // 2 for L in P.L_R[:2]],
              {k: f"{e:.1e}" for k, e in out.items()}, flush=True)
        del P
        torch.cuda.empty_cache()
