"""SURVEY §8(d) algorithmic bytes per right-hand side (fp32 unless s = 8), shared by the
measurement tools (passtime.py, pmc_cfg_summary.py, bench_configs.py).

* ``b_k``  — K / C^-1 on the reference's pruned-pass model (``8M + 32 m1 h2`` for d = 2 ...).
* ``b_rt`` — R^T / R on the reference's n-grid (``4M + 16 m1 h2 + 16 n1 h2 + 4M'`` for d = 2 ...):
  the figure ``roofline`` fractions of R / R^T are quoted against.
* ``floor_rt`` — the same pass structure on the grid the build actually transforms (``L_R`` per
  axis, ``L_R >= n + m - 1``): a lower bound of what the five / three passes must move,
  so ``traffic / floor_rt`` isolates wasted re-reads from the structural cost of the longer grid.
  The spectrum bytes (read once per RHS chunk) are returned separately.
"""


def _prod(v):
    p = 1
    for x in v:
        p *= x
    return p


def ngrid(dims):
    return [2 * m - 2 if m > 1 else 1 for m in dims]


def b_k(dims, s=4):
    d = len(dims)
    M = _prod(dims)
    c = 2 * s                       # complex
    if d == 1:
        return 2 * s * M
    n = ngrid(dims)
    h = dims[-1]                    # n_d / 2 + 1 = m_d
    if d == 2:
        return 2 * s * M + 4 * c * dims[0] * h
    return 2 * s * M + 4 * c * dims[0] * dims[1] * h + 4 * c * dims[0] * n[1] * h


def b_rt(dims, s=4):
    d = len(dims)
    M = _prod(dims)
    n = ngrid(dims)
    Mp = _prod(n)
    c = 2 * s
    if d == 1:
        return s * M + s * Mp
    h = dims[-1]
    if d == 2:
        return s * M + 2 * c * dims[0] * h + 2 * c * n[0] * h + s * Mp
    return (s * M + 2 * c * dims[0] * dims[1] * h + 2 * c * dims[0] * n[1] * h
            + 4 * c * n[0] * n[1] * h + s * Mp)


def floor_rt(dims, L_R, s=4, real_spec=True):
    """(bytes per RHS, spectrum bytes per chunk) of R^T on the L_R grid (compact last axis).
    L_R may carry trailing unit entries (hgp_plan_info pads it to three axes): they are dropped,
    so that the compact last axis is the grid's own last axis."""
    d = len(dims)
    L_R = list(L_R)
    if len(L_R) > d:
        assert all(v == 1 for v in L_R[d:]), L_R
        L_R = L_R[:d]
    M = _prod(dims)
    n = ngrid(dims)
    Mp = _prod(n)
    c = 2 * s
    hR = L_R[-1] // 2 + 1
    if d == 1:
        return s * M + s * Mp, (s if real_spec else c) * hR
    if d == 2:
        per = s * M + 2 * c * dims[0] * hR + 2 * c * n[0] * hR + s * Mp
        spec = (s if real_spec else c) * hR * L_R[0]
        return per, spec
    per = (s * M + 2 * c * dims[0] * dims[1] * hR + 2 * c * dims[0] * L_R[1] * hR
           + 2 * c * n[0] * L_R[1] * hR + 2 * c * n[0] * n[1] * hR + s * Mp)
    spec = (s if real_spec else c) * hR * L_R[1] * L_R[0]
    return per, spec


def op_bytes(op, dims, s=4):
    return b_rt(dims, s) if op in ("RT", "R") else b_k(dims, s)
