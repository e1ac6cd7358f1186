"""Grid-block (slab) sharding (row e2, hipgp_amd.slab) on the CPU with gloo: the axis-0 rows of
a 2-D / 3-D grid split over world_size 2 and 3 ranks, the passes of the reference's own operator
definition (tests/slab_cpu_engine.py), the all-to-all transposes and the all-reduced CG dots of
SlabToeplitz -- K, C^-1, R^T, R and the PCG (`cg.py:44-80`, break rule `cg.py:70`) gathered
from the ranks equal the single-process oracle."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import ziggy_oracle as zo

CASES = {"2d": ((13, 9), "matern", 1.5, (1., .3)), "3d": ((6, 5, 4), "sqexp", None, (1., .4)),
         "2d_long": ((4, 17), "matern", 2.5, (1., .5))}


def _oracle(case):
    dims, kind, nu, params = CASES[case]
    grids = [np.linspace(-1, 1, m) for m in dims]
    col = zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval(kind, x, y, params, nu=nu), 1e-2)
    return zo.ToeplitzOracle(col, dims)


def _worker(rank, ws, port, case, out, a2a_max=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from slab_cpu_engine import CpuSlabEngine
        from hipgp_amd import _lib
        from hipgp_amd import slab
        from hipgp_amd.slab import SlabToeplitz
        if a2a_max is not None:
            slab.A2A_MAX_BYTES = a2a_max     # exchanges in pieces (same count on every rank)
        T = _oracle(case)
        S = SlabToeplitz(T.dims, CpuSlabEngine(T))
        if a2a_max is not None:
            S.xchg_budget = 1                # and one right-hand side per exchange chunk
        rs = np.random.RandomState(4)
        v = torch.tensor(rs.randn(3, T.M))
        w = torch.tensor(rs.randn(3, T.Mp))
        res = {}
        for name, op, x, grid in (("K", _lib.OP_K, v, "m"), ("Cinv", _lib.OP_CINV, v, "m"),
                                  ("RT", _lib.OP_RT, v, "m"), ("R", _lib.OP_R, w, "n")):
            res[name] = S.apply(op, S.scatter_rows(x, grid)).numpy()
        x, it = S.pcg(S.scatter_rows(v), maxiter=8, tol=1e-8)
        res["pcg"], res["pcg_it"] = x.numpy(), it
        calls = []
        x2, it2 = S.pcg(S.scatter_rows(v), maxiter=200, tol=1e-3, callback=lambda n, xx: calls.append(n))
        res["brk"], res["brk_it"], res["brk_calls"] = x2.numpy(), it2, len(calls)
        res["kn"] = S.compute_kn(S.scatter_rows(v), maxiter=8, tol=1e-8).numpy()
        res["parts"] = sorted((op, b["parts_fwd"], b["parts_back"]) for op, b in S._buf.items())
        res["own_bytes"] = sorted((op, max(sum(b["sizes_in"]), sum(b["sizes_rx"])) * 16) for op, b in S._buf.items())
        out[rank] = res
    finally:
        dist.destroy_process_group()


def _gather(out, ws, key):
    return np.concatenate([out[r][key] for r in range(ws)], axis=1)


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("ws", [2, 3])
def test_slab_ops_and_pcg_gloo(case, ws):
    T = _oracle(case)
    rs = np.random.RandomState(4)
    v = rs.randn(3, T.M)
    w = rs.randn(3, T.Mp)
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29800 + os.getpid() % 150 + 10 * ws + len(case)
    mp.spawn(_worker, args=(ws, port, case, out), nprocs=ws, join=True)
    assert len(out) == ws
    for name, ref in (("K", T.matmul_K(v)), ("Cinv", T.matmul_Cinv(v)), ("RT", T.matmul_RT(v)), ("R", T.matmul_R(w))):
        got = _gather(out, ws, name)
        assert got.shape == ref.shape, name
        assert np.max(np.abs(got - ref)) <= 1e-11 * np.max(np.abs(ref)), name
    ref = T.solve(v, True, 8, 1e-8)
    assert np.max(np.abs(_gather(out, ws, "pcg") - ref)) <= 1e-9 * np.max(np.abs(ref))
    calls = []
    ref2 = T.solve(v, True, 200, 1e-3, callback=lambda n, x: calls.append(n))
    assert out[0]["brk_it"] == out[ws - 1]["brk_it"] == len(calls) + 1 < 200
    assert out[0]["brk_calls"] == len(calls)
    assert np.max(np.abs(_gather(out, ws, "brk") - ref2)) <= 1e-9 * np.max(np.abs(ref2))
    kn = zo.compute_kn(T, v, maxiter_cg=8, tol=1e-8)
    assert np.max(np.abs(_gather(out, ws, "kn") - kn)) <= 1e-9 * np.max(np.abs(kn))


def test_slab_split_exchanges_uneven_gloo():
    """Exchanges split into pieces (A2A_MAX_BYTES lowered to 256 bytes) with uneven row splits (13
    rows, 24 expanded rows over 3 ranks): every rank must issue the same number of pieces --
    the count comes from the largest rank's total, not the rank's own -- and the results stay
    the oracle's (hipgp_amd/slab.py a2a_parts).  The right-hand sides also go through
    the exchange one at a time (xchg_budget: the chunked apply, one shared arena)."""
    case, ws = "2d", 3
    T = _oracle(case)
    rs = np.random.RandomState(4)
    v = rs.randn(3, T.M)
    w = rs.randn(3, T.Mp)
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29700 + os.getpid() % 90
    mp.spawn(_worker, args=(ws, port, case, out, 256), nprocs=ws, join=True)
    assert len(out) == ws
    parts = [out[r]["parts"] for r in range(ws)]
    assert all(p == parts[0] for p in parts), parts
    assert all(pf > 1 and pb > 1 for _, pf, pb in parts[0]), parts[0]
    # the ranks' own totals differ (so a per-rank count could have differed)
    own = [dict(out[r]["own_bytes"]) for r in range(ws)]
    assert any(len({o[k] for o in own}) > 1 for k in own[0]), own
    for name, ref in (("K", T.matmul_K(v)), ("Cinv", T.matmul_Cinv(v)), ("RT", T.matmul_RT(v)), ("R", T.matmul_R(w))):
        got = _gather(out, ws, name)
        assert np.max(np.abs(got - ref)) <= 1e-11 * np.max(np.abs(ref)), name
    ref = T.solve(v, True, 8, 1e-8)
    assert np.max(np.abs(_gather(out, ws, "pcg") - ref)) <= 1e-9 * np.max(np.abs(ref))
