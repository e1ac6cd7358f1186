"""Diagnostic: plan dqf / column grads vs the oracle on small grids (GPU box)."""
import sys
sys.path[:0] = ["tests", "."]
import numpy as np
import torch
from golden_cases import rel_err
from oracle import ziggy_oracle as zo
from hipgp_amd import _lib
from hipgp_amd.plan import ToeplitzPlan

for dims in ((40,), (300,), (12, 10), (6, 5, 4)):
    M = int(np.prod(dims))
    rs = np.random.RandomState(0)
    l, r = rs.randn(2, M), rs.randn(2, M)
    P = ToeplitzPlan(dims, dtype=torch.float64, device="cuda")
    col = np.exp(-np.arange(M) / 5.0)
    P.set_column(torch.tensor(col, device="cuda"))
    got = P.dqf(torch.tensor(l, device="cuda"), torch.tensor(r, device="cuda")).cpu().numpy()
    want = zo.sym_toeplitz_dqf(l.T, r.T)
    print(dims, "dqf err %.2e" % rel_err(got, want), "got[:4]", got[:4], "want[:4]", want[:4], flush=True)
    T = zo.ToeplitzOracle(col, dims)
    for op, name, nin, nout in ((_lib.OP_K, "K", M, T.Mp if False else M), (_lib.OP_RT, "RT", M, T.Mp)):
        x, g = rs.randn(2, nin), rs.randn(2, nout)
        gg = P.column_grad(op, torch.tensor(x, device="cuda"), torch.tensor(g, device="cuda")).cpu().numpy()
        print("   ", name, "colgrad err %.2e" % rel_err(gg, T.column_grad(name, x, g)), flush=True)
