"""Diagnose fp64 3-D sweep failures: op errors vs the oracle, repeated, per shape (GPU box)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ziggy_oracle as zo  # noqa: E402


def main():
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    shapes = [(5, 40, 2), (129, 3, 2), (2, 2, 2), (4, 40, 2), (5, 2, 2), (5, 40, 3), (5, 40, 4), (5, 8, 2), (64, 64, 2)]
    for dt in (torch.float64, torch.float32):
        for dims in shapes:
            grids = [np.linspace(-1, 1, m) for m in dims]
            col = zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., 4.0 / max(dims)), nu=1.5), 0.05)
            O = zo.ToeplitzOracle(col, dims)
            P = ToeplitzPlan(dims, dt, "cuda")
            P.set_column(torch.tensor(col, device="cuda", dtype=dt))
            v = np.random.RandomState(1).randn(3, O.M)
            vt = torch.tensor(v, device="cuda", dtype=dt)
            errs = []
            for op, ref in ((_lib.OP_K, O.matmul_K(v)), (_lib.OP_CINV, O.matmul_Cinv(v))):
                for _ in range(3):
                    got = P.apply(op, vt).double().cpu().numpy()
                    errs.append(float(np.abs(got - ref).max() / np.abs(ref).max()))
                one = P.apply(op, vt[:1]).double().cpu().numpy()
                errs.append(float(np.abs(one - ref[:1]).max() / np.abs(ref[:1]).max()))
            print(str(dt)[-7:], dims, " ".join("%.1e" % e for e in errs), flush=True)


if __name__ == "__main__":
    main()
