"""CPU oracle of the backward vs the reference's own gradients
(golden vectors G13-G15: InvMatmul.backward's column / right-hand-side gradients and the
column gradients of R^T, K, C^-1, R through the spectrum, made by autograd on the reference)."""
import numpy as np
import pytest

from golden_cases import load, rel_err
from grad_cases import GRAD_CASES, GRAD_MAXITER, GRAD_TOL
from oracle import ziggy_oracle as zo


def _oracle(fx):
    dims = tuple(int(d) for d in fx["dims"])
    return zo.ToeplitzOracle(fx["column"].astype(np.float64), dims)


@pytest.mark.parametrize("name", sorted(GRAD_CASES))
def test_inv_matmul_backward_oracle(name):
    fx = load(name, "f64")
    T = _oracle(fx)
    cg, left = zo.inv_matmul_column_grad(T, fx["solves"], fx["grad_out"], GRAD_MAXITER, GRAD_TOL)
    # G14 (SqExp, cond ~1e7): the two fp64 PCGs agree to ~4e-7 after 30 iterations
    tol = 2e-6 if name == "G14" else 1e-10
    assert rel_err(cg, fx["inv_column_grad"]) < tol
    assert rel_err(left, fx["inv_right_grad"]) < tol


@pytest.mark.parametrize("name", sorted(GRAD_CASES))
@pytest.mark.parametrize("op", ["RT", "K", "Cinv", "R"])
def test_operator_column_grad_oracle(name, op):
    fx = load(name, "f64")
    T = _oracle(fx)
    x, g, ref = (fx["rt_v"], fx["rt_g"], fx["rt_column_grad"]) if op == "RT" else \
        (fx[f"{op}_x"], fx[f"{op}_g"], fx[f"{op}_column_grad"])
    assert rel_err(T.column_grad(op, x, g), ref) < 1e-10


def test_dqf_definition():
    """The lag-sum definition (`gpt_toeplitz.py:169-209` docstring) on random vectors,
    including n = 1 and ragged n."""
    rs = np.random.RandomState(3)
    for n, s in ((1, 2), (5, 1), (37, 3), (300, 2)):
        l, r = rs.randn(n, s), rs.randn(n, s)
        want = np.zeros(n)
        for i in range(n):
            for j in range(s):
                T = np.eye(n, k=i) + np.eye(n, k=-i) if i else np.eye(n)
                want[i] += l[:, j] @ T @ r[:, j]
        assert rel_err(zo.sym_toeplitz_dqf(l, r), want) < 1e-12
