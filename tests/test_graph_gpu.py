"""Repeated hgp_toeplitz_apply calls replay a captured hipGraph (the second identical call is
captured, later ones launch the graph): results are bitwise those of direct launches (a plan
created with HGP_GRAPH=0), across ops, 2-D / 3-D, chunked RHS on two streams, and after the
arguments, the workspace or the stream change."""
import os

import numpy as np
import pytest
import torch

from oracle import ziggy_oracle as zo

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _plans(dims, dt):
    from hipgp_amd.plan import ToeplitzPlan
    grids = [np.linspace(-1, 1, m) for m in dims]
    col = torch.tensor(zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("sqexp", x, y, (1., .2)), 1e-2),
                       device=DEV, dtype=dt)
    P = ToeplitzPlan(dims, dt, DEV)
    P.set_column(col)
    os.environ["HGP_GRAPH"] = "0"
    try:
        Q = ToeplitzPlan(dims, dt, DEV)
    finally:
        del os.environ["HGP_GRAPH"]
    Q.set_column(col)
    return P, Q


@pytest.mark.parametrize("dims,dt", [((96, 80), torch.float32), ((40, 24, 20), torch.float64), ((1024, 1024), torch.float32)],
                         ids=["2d_f32", "3d_f64", "C2_f32"])
def test_graph_replay_bitwise(dims, dt):
    from hipgp_amd import _lib
    P, Q = _plans(dims, dt)
    M = int(np.prod(dims))
    Mp = int(np.prod([2 * m - 2 for m in dims]))
    g = torch.Generator(device=DEV).manual_seed(5)
    for nrhs in (3, 17):
        x = torch.randn(nrhs, M, device=DEV, generator=g, dtype=dt)
        w = torch.randn(nrhs, Mp, device=DEV, generator=g, dtype=dt)
        for op, v in ((_lib.OP_K, x), (_lib.OP_CINV, x), (_lib.OP_RT, x), (_lib.OP_R, w)):
            ref = Q.apply(op, v)
            y = torch.empty_like(ref)
            for rep in range(4):                   # direct, captured, replayed, replayed
                y.zero_()
                P.apply(op, v, out=y)
                assert torch.equal(y, ref), (op, nrhs, rep)
            v2 = v * 2                              # new input buffer: not the captured graph
            assert torch.equal(P.apply(op, v2), Q.apply(op, v2)), (op, "new args")
    # a new stream: the plan rebinds, the cached graph (other stream) is not replayed
    s = torch.cuda.Stream(device=DEV)
    with torch.cuda.stream(s):
        y = torch.empty_like(x)
        for _ in range(3):
            P.apply(_lib.OP_K, x, out=y)
        ref = Q.apply(_lib.OP_K, x)
    s.synchronize()
    assert torch.equal(y, ref)


def test_graph_key_tracks_plan_buffers():
    """on a plan with an axis beyond 8192 points every operator runs the
    full-grid route in gridA / gridB, sized to prod(L_K) for K and prod(L_R) for R^T.  K, K (the
    second call is captured), R^T (grows and so reallocates both buffers), then K again with the
    SAME x / y: the graph key holds every plan buffer an op addresses, so the last K runs
    directly again instead of replaying a graph on the freed buffers -- its result equals a
    graph-free plan's bit for bit."""
    from hipgp_amd import _lib
    dims = (5, 12000)
    P, Q = _plans(dims, torch.float32)
    M = int(np.prod(dims))
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.randn(2, M, device=DEV, generator=g)
    y = torch.empty_like(x)
    ref = Q.apply(_lib.OP_K, x)
    for _ in range(2):                            # direct, then captured
        P.apply(_lib.OP_K, x, out=y)
        assert torch.equal(y, ref)
    rt = P.apply(_lib.OP_RT, x)                   # full-grid buffers regrown for L_R
    assert torch.equal(rt, Q.apply(_lib.OP_RT, x))
    for _ in range(3):                            # K with the captured call's x / y again
        y.fill_(float("nan"))
        P.apply(_lib.OP_K, x, out=y)
        torch.cuda.synchronize()
        assert torch.equal(y, ref)
