"""Grid-block (slab) sharding of the Toeplitz operators and the PCG over ranks (row e2).

`north_star`: "independent grid blocks shard across the 8 GPUs ... RCCL all-reduce of CG
dot-products"; BASELINE config 5 is a "grid-block shard on 8xMI355X".  Where the RHS split of
`hipgp_amd.dist` gives every rank whole right-hand sides, here every rank owns a block of
axis-0 rows of EVERY right-hand side (a slab of the 2-D / 3-D grid):

* the per-axis passes along the other axes (`toeplitz_tensor.py:79,94,109,122` restated as
  the library's pruned row / middle-axis transforms) are local to the slab;
* the axis-0 convolution needs whole axis-0 lines: an all-to-all transposes the exchange
  layout E[g][q][i][c] (hgp_slab_pass, include/hipgp.h) from "my rows, all groups" to "all
  rows, my groups", the convolution runs on the rank's groups, and a second all-to-all brings
  the result back;
* every CG scalar of `cg.py:64,66,69,74` becomes a sum of per-rank partial dots: one
  all-reduce(SUM) of B values per dot (p.Ap, r.r, z.r: three per iteration), and the all-RHS
  break rule `cg.py:70` is decided on the reduced r.r, identically on every rank.

Backend: "nccl" (= RCCL over xGMI) on GPUs; "gloo" (tests, same-device rehearsals) stages
CUDA tensors through the host.  The pass engine is libhipgp (HipSlabEngine); the CPU tests
plug in a NumPy engine with the same E layout contract.
"""
import ctypes

import torch
import torch.distributed as dist

from . import _lib
from ._lib import check, lib


def split(n, parts, k):
    """Contiguous balanced block k of range(n) over `parts` ranks: (start, stop)."""
    base, extra = divmod(n, parts)
    start = k * base + min(k, extra)
    return start, start + base + (1 if k < extra else 0)


# largest all-to-all handed to RCCL in one call.  Measured (tools/a2a_limit.py, world size 1,
# profiles/r6_a2a_limit_probe{1,2}.jsonl): one all_to_all_single of up to 1024 MiB is exact; from
# 1025 MiB on, for float32 and float64 alike and with or without explicit split sizes, every byte
# from about the middle of the buffer to its end comes back wrong -- a BYTE-count limit of 2^30
# in the RCCL self-exchange path (round 5 met it as a 2.4 GB config-5 R^T exchange).  Larger
# exchanges therefore go in pieces of at most 2^30 bytes (a2a_parts, the same count on every rank)
A2A_MAX_BYTES = 1 << 30


def a2a_parts(totals_bytes):
    """Number of pieces an exchange is split into.  `totals_bytes`: every rank's send and
    receive totals of this exchange.  It must be the SAME on every rank -- a rank that issued
    one all-to-all while a peer issued several would hang or pair mismatched pieces -- so it
    comes from the largest total of any rank, which every rank computes from the shared
    partition (SlabToeplitz._geom), never from its own byte count alone."""
    biggest = max([0] + [int(t) for t in totals_bytes])
    return max(1, -(-biggest // A2A_MAX_BYTES))


def _pieces(t, offs, sizes, j, parts):
    """Piece j (of `parts`) of every peer block [a, a + s) of the flat tensor t: contiguous views."""
    return [t[a + s * j // parts:a + s * (j + 1) // parts] for a, s in zip(offs, sizes)]


def _a2a(out, inp, out_splits, in_splits, group, parts=1):
    """all_to_all_single on real views (complex / CUDA through the host for gloo), in `parts`
    pieces (a2a_parts: the same count on every rank): piece j moves the j-th equal part of every
    peer's block.  RCCL takes the pieces as list all-to-alls over views (no copies); gloo, which
    has no list all-to-all, packs each piece of its host copy into one all_to_all_single."""
    gloo = dist.get_backend(group) == "gloo"
    i = torch.view_as_real(inp).reshape(-1) if inp.is_complex() else inp.reshape(-1)
    o = torch.view_as_real(out).reshape(-1) if out.is_complex() else out.reshape(-1)
    f = 2 if inp.is_complex() else 1
    so, si = [f * s for s in out_splits], [f * s for s in in_splits]
    oo = [sum(so[:r]) for r in range(len(so))]
    oi = [sum(si[:r]) for r in range(len(si))]
    if gloo:
        ih = i.cpu()
        oh = torch.empty(o.shape, dtype=o.dtype) if o.is_cuda else o
        if parts == 1:
            dist.all_to_all_single(oh, ih, so, si, group=group)
        else:
            for j in range(parts):
                src = _pieces(ih, oi, si, j, parts)
                dst = _pieces(oh, oo, so, j, parts)
                buf = torch.empty(sum(d.numel() for d in dst), dtype=oh.dtype)
                dist.all_to_all_single(buf, torch.cat(src), [d.numel() for d in dst], [p.numel() for p in src],
                                       group=group)
                k = 0
                for d in dst:
                    d.copy_(buf[k:k + d.numel()])
                    k += d.numel()
        if oh is not o:
            o.copy_(oh)
        return out
    if parts == 1:
        dist.all_to_all_single(o, i, so, si, group=group)
        return out
    for j in range(parts):
        dist.all_to_all(_pieces(o, oo, so, j, parts), _pieces(i, oi, si, j, parts), group=group)
    return out


def _allreduce(t, group):
    if dist.get_backend(group) == "gloo" and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


class HipSlabEngine:
    """The slab stages on libhipgp (hgp_slab_pass_ex), one replicated plan per rank, and the
    slab PCG's vector / scalar updates (hgp_slab_cg_*) on device buffers."""

    def __init__(self, plan):
        self.plan = plan
        self.dtype = plan.dtype
        self.cdtype = torch.complex64 if plan.dtype == torch.float32 else torch.complex128
        self.device = plan.device
        if len(plan.dims) - sum(1 for m in plan.dims if m == 1) < 2:
            raise _lib.HipgpError("slab sharding needs a 2-D or 3-D grid")

    def geometry(self, op):
        ng, inner = ctypes.c_int64(), ctypes.c_int64()
        check(lib().hgp_slab_info(self.plan._h, int(op), ctypes.byref(ng), ctypes.byref(inner)))
        return ng.value, inner.value

    @staticmethod
    def _p(t):
        return ctypes.c_void_p(None if t is None else t.data_ptr())

    def _run(self, op, stage, x, y, nrhs, nrows, g0=0, ng=0, dotv=None, dot_out=None, done=None):
        self.plan._bind_stream()
        check(lib().hgp_slab_pass_ex(self.plan._h, int(op), int(stage), self._p(x), self._p(y), nrhs, nrows, g0, ng,
                                     self._p(dotv), self._p(dot_out), self._p(done)))

    def fwd(self, op, x, nrows, E, done=None):
        self._run(op, _lib.SLAB_FWD, x.contiguous(), E, x.shape[0], nrows, done=done)

    def conv(self, op, lines, g0, ng, nrhs):
        self._run(op, _lib.SLAB_CONV, lines, lines, nrhs, 0, g0, ng)

    def conv_a2a(self, op, recv, send, g0, ng, nrhs, ws, done=None):
        self._run(op, _lib.SLAB_CONV_A2A, recv, send, nrhs, ws, g0, ng, done=done)

    def inv(self, op, E, nrows, y, dotv=None, dot_out=None, done=None):
        self._run(op, _lib.SLAB_INV, E, y, y.shape[0], nrows, dotv=dotv, dot_out=dot_out, done=done)

    # -- slab PCG updates (cg.py:63-78); dots already all-reduced; no-ops once done ----------
    def dot(self, a, c, out):
        if a.shape[1] == 0:
            out.zero_()
            return
        check(lib().hgp_rowdot(_lib.dtype_code(a.dtype), self._p(a), self._p(c), self._p(out), a.shape[0],
                               a.shape[1], _lib.stream_ptr(a.device)))

    def cg_xr(self, x, r, p, Ap, rs, pAp, rr, done):
        self.plan._bind_stream()
        check(lib().hgp_slab_cg_xr(self.plan._h, self._p(x), self._p(r), self._p(p), self._p(Ap), self._p(rs),
                                   self._p(pAp), self._p(rr), x.shape[0], x.shape[1], self._p(done)))

    def cg_check(self, rr, tol, done, iters):
        self.plan._bind_stream()
        check(lib().hgp_slab_cg_check(self.plan._h, self._p(rr), rr.shape[0], float(tol), self._p(done),
                                      self._p(iters)))

    def cg_p(self, p, z, rs, zr, done):
        self.plan._bind_stream()
        check(lib().hgp_slab_cg_p(self.plan._h, self._p(p), self._p(z), self._p(rs), self._p(zr), p.shape[0],
                                  p.shape[1], self._p(done)))


class SlabToeplitz:
    """K, C^-1, R^T, R (`toeplitz_tensor.py:70-125`) of a 2-D / 3-D grid whose axis-0 rows are
    split over the ranks of `group`.  dims: the m-grid; vectors on the m-grid are local slabs
    (nrhs, rows_m(rank) * prod(dims[1:])), on the expanded n-grid (R input, R^T output)
    (nrhs, rows_n(rank) * prod(n[1:]))."""

    def __init__(self, dims, engine, group=None):
        self.engine = engine
        self.group = group
        self.ws = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        dims = tuple(int(m) for m in dims if int(m) > 1)
        if len(dims) < 2:
            raise ValueError("slab sharding needs at least two axes with more than one point")
        self.dims = dims
        self.ndims = tuple(2 * m - 2 for m in dims)
        self.rest_m = 1
        self.rest_n = 1
        for a in range(1, len(dims)):
            self.rest_m *= dims[a]
            self.rest_n *= self.ndims[a]
        self.rows_m = [split(dims[0], self.ws, k) for k in range(self.ws)]
        self.rows_n = [split(self.ndims[0], self.ws, k) for k in range(self.ws)]
        self._buf = {}
        self._arena = None
        import os
        self.xchg_budget = int(os.environ.get("HGP_SLAB_XCHG_MB", "4096")) << 20

    # -- partition ------------------------------------------------------------------------
    def my_rows(self, grid="m"):
        return (self.rows_m if grid == "m" else self.rows_n)[self.rank]

    def local_size(self, grid="m"):
        a, b = self.my_rows(grid)
        return (b - a) * (self.rest_m if grid == "m" else self.rest_n)

    def scatter_rows(self, v, grid="m"):
        """This rank's slab of full vectors v (nrhs, M or M')."""
        a, b = self.my_rows(grid)
        rest = self.rest_m if grid == "m" else self.rest_n
        return v[:, a * rest:b * rest].contiguous()

    # -- the operator ---------------------------------------------------------------------
    def _check(self, t, name, grid, nrhs=None):
        """t must be this rank's contiguous slab (nrhs, local size of `grid`) in the engine's dtype
        on its device: the engine hands raw pointers to the library, which dispatches on the
        plan's dtype and trusts the sizes."""
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"{name} must be a tensor")
        if t.dtype != self.engine.dtype:
            raise TypeError(f"{name} has dtype {t.dtype}, the slab plan is {self.engine.dtype}")
        dev = getattr(self.engine, "device", None)
        if dev is not None and t.device != torch.device(dev):
            raise ValueError(f"{name} is on {t.device}, the slab plan on {dev}")
        size = self.local_size(grid)
        if t.dim() != 2 or t.shape[1] != size or (nrhs is not None and t.shape[0] != nrhs):
            want = f"({'nrhs' if nrhs is None else nrhs}, {size})"
            raise ValueError(f"{name} must be this rank's slab {want}, got {tuple(t.shape)}")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
        return t

    def _geom(self, op, nrhs):
        """The exchange geometry of (op, nrhs) (cached; no tensors): group split, row counts, the
        two all-to-alls' split sizes and piece counts, element counts of the buffers."""
        key = (int(op), int(nrhs))
        b = self._buf.get(key)
        if b is None:
            ws, rk = self.ws, self.rank
            rows_in = self.rows_n if op == _lib.OP_R else self.rows_m
            rows_out = self.rows_n if op == _lib.OP_RT else self.rows_m
            NG, inner = self.engine.geometry(op)
            groups = [split(NG, ws, k) for k in range(ws)]
            gs0, gs1 = groups[rk]
            ng = gs1 - gs0
            ni = rows_in[rk][1] - rows_in[rk][0]
            no = rows_out[rk][1] - rows_out[rk][0]
            # E[g][q][i][c] over my input rows; the first all-to-all sends my rows of every group
            # and receives all rows of my groups as rank blocks [r][g][q][i - a_r][c] (rank r's
            # rows [a_r, a_r + cnt_r)); the conv writes the return all-to-all's send buffer as
            # rank blocks [r][g][q][o - b_r][c] (HGP_SLAB_CONV_A2A: no line buffer, no gather /
            # scatter copies); the return all-to-all delivers my output rows of every group
            cnt = lambda rows, r: rows[r][1] - rows[r][0]
            gcnt = lambda r: groups[r][1] - groups[r][0]

            def sizes(r):    # rank r's (sizes_in, sizes_rx, sizes_tx, sizes_back), in elements
                return ([gcnt(s) * nrhs * cnt(rows_in, r) * inner for s in range(ws)],
                        [gcnt(r) * nrhs * cnt(rows_in, s) * inner for s in range(ws)],
                        [gcnt(r) * nrhs * cnt(rows_out, s) * inner for s in range(ws)],
                        [gcnt(s) * nrhs * cnt(rows_out, r) * inner for s in range(ws)])
            sizes_in, sizes_rx, sizes_tx, sizes_back = sizes(rk)
            # piece counts of the two exchanges from EVERY rank's totals (a2a_parts): identical
            # on all ranks even where uneven splits put the ranks' own totals on either side of
            # a multiple of A2A_MAX_BYTES
            esz = self._csize()
            every = [sizes(r) for r in range(ws)]
            parts_fwd = a2a_parts([sum(v) * esz for e in every for v in (e[0], e[1])])
            parts_back = a2a_parts([sum(v) * esz for e in every for v in (e[2], e[3])])
            nE, nback = NG * nrhs * ni * inner, NG * nrhs * no * inner
            b = dict(nrhs=int(nrhs), NG=NG, inner=inner, gs0=gs0, ng=ng, ni=ni, no=no, sizes_in=sizes_in,
                     sizes_rx=sizes_rx, sizes_tx=sizes_tx, sizes_back=sizes_back, parts_fwd=parts_fwd,
                     parts_back=parts_back, nE=nE, nback=nback, nrecv=sum(sizes_rx), nsend=sum(sizes_tx))
            self._buf[key] = b
        return b

    def _csize(self):
        return torch.empty((), dtype=self.engine.cdtype).element_size()

    def xchg_bytes_per_rhs(self, op):
        """Device bytes of one apply's exchange buffers per right-hand side."""
        b = self._geom(op, 1)
        return (max(b["nE"], b["nback"]) + b["nrecv"] + b["nsend"]) * self._csize()

    def _arena_views(self, b, dev):
        """The buffers of one apply as views of ONE arena shared by every op and chunk (applies
        run one after another on the stream; nothing in them outlives the apply):
        [E | back] (E is consumed by the first all-to-all before the second one writes back, so
        they share storage) + recv + send.  The arena grows to the largest apply and is
        allocated once: a PCG iteration allocates nothing."""
        cd = self.engine.cdtype
        n0 = max(b["nE"], b["nback"])
        need = n0 + b["nrecv"] + b["nsend"]
        a = self._arena
        if a is None or a.numel() < need or a.device != torch.device(dev):
            self._arena = a = None
            self._arena = a = torch.empty(need, dtype=cd, device=dev)
        E = a[:b["nE"]].view(b["NG"], b["nrhs"], b["ni"], b["inner"])
        back = a[:b["nback"]]
        recv = a[n0:n0 + b["nrecv"]]
        send = a[n0 + b["nrecv"]:need]
        return E, back, recv, send

    def release(self):
        """Drop the exchange arena (re-allocated on the next apply)."""
        self._buf.clear()
        self._arena = None

    def apply(self, op, x, out=None, dotv=None, dot_out=None, done=None):
        """op (libhipgp OP_*) on this rank's slab x (nrhs, local in-size) -> local out slab
        (written into `out` when given).  dotv / dot_out: also this rank's per-RHS dots
        sum(out * dotv) (fused into the last stage); done: a device flag after which every
        stage is a no-op (the slab PCG's masked iterations).

        The right-hand sides go through the exchange in chunks of at most `xchg_budget` bytes of
        buffers (default HGP_SLAB_XCHG_MB = 4096), so the device memory of the exchange does not
        grow with the batch (config 5's R^T at B = 25 would need 19 GB in one piece); every rank
        has the same chunking (the geometry is shared), so the collectives line up."""
        x = self._check(x.contiguous(), "x", "n" if op == _lib.OP_R else "m")
        nrhs = x.shape[0]
        if out is not None:
            self._check(out, "out", "n" if op == _lib.OP_RT else "m", nrhs)
        if dotv is not None:
            self._check(dotv, "dotv", "n" if op == _lib.OP_RT else "m", nrhs)
        if dot_out is not None and (dot_out.dtype != x.dtype or dot_out.numel() != nrhs
                                    or not dot_out.is_contiguous() or dot_out.device != x.device):
            raise ValueError(f"dot_out must be a contiguous ({nrhs},) {x.dtype} vector on {x.device}")
        rest_out = self.rest_n if op == _lib.OP_RT else self.rest_m
        y = torch.empty((nrhs, self.local_size("n" if op == _lib.OP_RT else "m")), dtype=x.dtype,
                        device=x.device) if out is None else out
        if nrhs == 0:
            return y
        qc = max(1, min(nrhs, int(self.xchg_budget // max(1, self.xchg_bytes_per_rhs(op)))))
        for q0 in range(0, nrhs, qc):
            q1 = min(nrhs, q0 + qc)
            self._apply_chunk(op, x[q0:q1], y[q0:q1], None if dotv is None else dotv[q0:q1],
                              None if dot_out is None else dot_out[q0:q1], done, rest_out)
        return y

    def _apply_chunk(self, op, x, y, dotv, dot_out, done, rest_out):
        e = self.engine
        nrhs = x.shape[0]
        b = self._geom(op, nrhs)
        E, back, recv, send = self._arena_views(b, x.device)
        ni, no, ng = b["ni"], b["no"], b["ng"]
        # 1. local transforms along the other axes over my input rows
        if ni > 0:
            e.fwd(op, x, ni, E, done=done)
        # 2. all-to-all: my rows of every group -> all rows of my groups
        _a2a(recv, E.reshape(-1), b["sizes_rx"], b["sizes_in"], self.group, b["parts_fwd"])
        # 3. the axis-0 convolution of my groups, receive buffer -> send buffer
        if ng > 0:
            e.conv_a2a(op, recv, send, b["gs0"], ng, nrhs, self.ws, done=done)
        # 4. all-to-all back: all rows of my groups -> my output rows of every group (into E's storage)
        _a2a(back, send, b["sizes_back"], b["sizes_tx"], self.group, b["parts_back"])
        E2 = back.view(b["NG"], nrhs, no, b["inner"])      # groups arrive in rank order = group order
        # 5. local inverse transforms over my output rows (+ fused dot)
        if no > 0:
            e.inv(op, E2, no, y, dotv=dotv, dot_out=dot_out, done=done)
        elif dot_out is not None:
            dot_out.zero_()

    # -- PCG -------------------------------------------------------------------------------
    def dot(self, a, b):
        """Global per-RHS dot products: local row sums, one all-reduce of nrhs values."""
        s = torch.empty(a.shape[0], dtype=a.dtype, device=a.device)
        self.engine.dot(a, b, s)
        return _allreduce(s, self.group)

    def pcg(self, b, maxiter=20, tol=1e-8, precond=True, callback=None):
        """conj_grad2 (`cg.py:44-80`) on the slabs: x0 = 0, per-RHS alpha / beta from all-reduced
        dots, break when EVERY global sqrt(r.r) < tol.  Returns (x, iterations run).

        Per iteration: Ap = K p with the local p.Ap fused into its last stage; all-reduce;
        alpha, x += alpha p, r -= alpha Ap and the local r.r in one update (hgp_slab_cg_xr);
        all-reduce; the break test on the reduced r.r (identical on every rank: a device flag
        `done` holding the iteration it fired in, hgp_slab_cg_check); z = C^-1 r with z.r fused;
        all-reduce; beta, rs and p = z + beta p (hgp_slab_cg_p).  Every kernel of the operators
        and updates is a no-op once `done` is set, so the host queues all `maxiter` iterations
        without a synchronisation (RCCL: the all-reduces / all-to-alls are stream-ordered) and
        the iterations after the break cost their (stale) collectives only; x is the iterate
        the reference's break returns.  Vectors, scalars and exchange buffers are allocated
        before the loop.  With a callback (`cg.py:77-78`, after every iteration that did not
        break) the host must look at the flag, so that form synchronises per iteration."""
        e = self.engine
        b = self._check(b.contiguous(), "b", "m")
        nrhs = b.shape[0]
        x = torch.zeros_like(b)
        r = b.clone()
        z = torch.empty_like(b) if precond else r
        Ap = torch.empty_like(b)
        sc = torch.zeros((4, nrhs), dtype=b.dtype, device=b.device)
        rs, pAp, rr, zr = sc[0], sc[1], sc[2], sc[3]
        flags = torch.zeros(2, dtype=torch.int32, device=b.device)
        done, iters = flags[0:1], flags[1:2]
        if precond:
            self.apply(_lib.OP_CINV, r, out=z, dotv=r, dot_out=rs)     # z0 = P r, rs = z.r
        else:
            e.dot(r, r, rs)
        _allreduce(rs, self.group)
        p = z.clone()
        for n in range(int(maxiter)):
            self.apply(_lib.OP_K, p, out=Ap, dotv=p, dot_out=pAp, done=done)
            _allreduce(pAp, self.group)
            e.cg_xr(x, r, p, Ap, rs, pAp, rr, done)
            _allreduce(rr, self.group)
            e.cg_check(rr, tol, done, iters)
            if callback is not None and int(done.item()):
                break
            if precond:
                self.apply(_lib.OP_CINV, r, out=z, dotv=r, dot_out=zr, done=done)
                _allreduce(zr, self.group)
                e.cg_p(p, z, rs, zr, done)
            else:
                e.cg_p(p, r, rs, rr, done)
            if callback is not None:
                callback(n, x)
        return x, int(iters.item())

    def compute_kn(self, Knm_local, maxiter=20, tol=1e-8):
        """kn = R^T K^{-1} Knm^T (`hipgp.py:143-145`) with Knm's axis-0 rows on this rank;
        returns this rank's rows of the expanded n-grid (nrhs, local M')."""
        d0, _ = self.pcg(Knm_local, maxiter, tol, precond=True)
        return self.apply(_lib.OP_RT, d0)


def slab_toeplitz(dims, column, dtype=torch.float32, device=None, group=None, jitter=0.0, clamp_min=1e-6):
    """SlabToeplitz on libhipgp: every rank builds the (replicated) spectrum of the whole grid
    from the full first row `column` (M,) and owns its axis-0 slab of every vector."""
    from .plan import ToeplitzPlan
    plan = ToeplitzPlan(dims, dtype=dtype, device=device)
    plan.set_column(column, jitter=jitter, clamp_min=clamp_min)
    return SlabToeplitz(dims, HipSlabEngine(plan), group=group)


def _all_gather_cols(local, group):
    """Concatenate the ranks' column blocks (nrhs, n_r) -> (nrhs, sum n_r) in rank order (the
    slabs' axis-0 row blocks are contiguous column ranges of the flattened grid).  Blocks may
    differ in width (balanced splits): each is padded to the widest, gathered, trimmed."""
    ws = dist.get_world_size(group)
    widths = torch.tensor([local.shape[1]], dtype=torch.int64)
    wl = [torch.zeros(1, dtype=torch.int64) for _ in range(ws)]
    if dist.get_backend(group) == "gloo":
        dist.all_gather(wl, widths, group=group)
    else:
        wd = widths.to(local.device)
        wg = [torch.zeros(1, dtype=torch.int64, device=local.device) for _ in range(ws)]
        dist.all_gather(wg, wd, group=group)
        wl = [w.cpu() for w in wg]
    wmax = max(int(w) for w in wl)
    pad = local.new_zeros((local.shape[0], wmax))
    pad[:, :local.shape[1]] = local
    gloo = dist.get_backend(group) == "gloo" and pad.is_cuda
    src = pad.cpu() if gloo else pad
    parts = [torch.empty_like(src) for _ in range(ws)]
    dist.all_gather(parts, src, group=group)
    full = torch.cat([p[:, :int(w)] for p, w in zip(parts, wl)], dim=1)
    return full.to(local.device) if gloo else full


class SlabKmm:
    """Grid-block sharding behind the reference's duck-typed `Kmm` (`hipgp.py:117-146`:
    `compute_kn(Knm, maxiter_cg, tol, Kmm=...)` needs `.inv_matmul(R, do_precond, maxiter, tol)`
    and `._matmul_by_RT(d)`), so an unchanged model can run its solve grid-block sharded
    (BASELINE config 5: "grid-block shard").

    Every rank of `group` passes the SAME full minibatch rows: `inv_matmul` takes the rank's
    axis-0 slab of R (B, M), runs the slab PCG (`SlabToeplitz.pcg`: all-reduced per-RHS dots,
    the all-rank break rule) and all-gathers the solution to (B, M) like ToeplitzTensor's;
    `_matmul_by_RT` applies R^T on the slabs (all-to-all transposes) and all-gathers the
    expanded-grid rows, so the caller gets the full (B, M') kn.  Forward only: the solve is not
    differentiable here (kernel-hyperparameter learning goes through the RHS-sharded
    `hipgp_amd.dist` path)."""

    def __init__(self, slab, column=None):
        self.slab = slab
        self.column = column
        self.dims = slab.dims
        self.ndim = len(slab.dims)
        self.M = int(slab.rest_m * slab.dims[0])

    @classmethod
    def from_model(cls, model, group=None):
        """The grid-block Kmm of a Toeplitz model's current kernel parameters: every rank sets
        the spectrum of the whole grid (replicated, as `model.toeplitz()` would) and owns its
        axis-0 slab of every vector."""
        T = model.toeplitz()
        T._plan.trim()                         # the set-up's fp64 transform buffers (GBs at C5)
        return cls(SlabToeplitz(T.dims, HipSlabEngine(T._plan), group=group), column=T.column)

    def set_batch_shape(self, batch_shape):
        self.batch_shape = tuple(batch_shape)

    def _check_grad(self, t):
        if torch.is_grad_enabled() and t.requires_grad:
            raise NotImplementedError("SlabKmm is forward-only: differentiate through the RHS-sharded path "
                                      "(hipgp_amd.dist.sharded_compute_kn) instead")

    def inv_matmul(self, right_tensor, do_precond=True, maxiter=20, tol=1e-8):
        """K^-1 R for the full rows R (B, M) (`toeplitz_tensor.py:47-52`), solved on the slabs."""
        self._check_grad(right_tensor)
        with torch.no_grad():
            x, _ = self.slab.pcg(self.slab.scatter_rows(right_tensor.contiguous(), "m"), maxiter, tol,
                                 precond=do_precond)
            return _all_gather_cols(x, self.slab.group)

    def _matmul_by_RT(self, vec):
        """R^T d for the full rows d (B, M) -> the full expanded-grid rows (B, M')
        (`toeplitz_tensor.py:85-97`)."""
        self._check_grad(vec)
        with torch.no_grad():
            y = self.slab.apply(_lib.OP_RT, self.slab.scatter_rows(vec.contiguous(), "m"))
            return _all_gather_cols(y, self.slab.group)


class SlabFit:
    """One natural-gradient minibatch of a mean-field model with the inducing grid split into
    axis-0 slabs over the ranks of `group` and kn KEPT in slabs (`hipgp.py:194-276` with the
    solve of `hipgp.py:117-146` on SlabToeplitz): per minibatch every rank

    * evaluates only its slab's Knm columns (`_make_grams(grid_rows=...)`: the fused Kuf kernels
      on the sub-grid xgrids[0][a:b] -- point or line-integral observations; the MC estimator's
      offset is drawn once and broadcast, `hipgp_amd.dist.shared_mc_offset`);
    * runs the slab PCG and R^T (`SlabToeplitz.compute_kn`): kn stays (B, its M' slab);
    * forms the statistics from B-length all-reduced dot partials and its own columns
      (`MeanFieldToeplitzGP.batch_stats_slab`), summed once over the ranks (`allreduce_stats`:
      2 M' values), after which every rank takes the same natural-gradient step.

    Nothing of size B x M' is gathered (the `SlabKmm` adapter behind `compute_kn(Kmm=)` gathers
    d and kn to full rows on every rank); per rank the minibatch holds B x M'/ws of kn.  The
    plan (spectra of the whole grid, replicated) and the exchange buffers are built once per fit:
    the grid mode runs with fixed kernel hyper-parameters."""

    def __init__(self, model, group=None, slab=None):
        if getattr(model, "name", None) != "mean-field" or not hasattr(model, "batch_stats_slab"):
            raise NotImplementedError("SlabFit keeps kn in slabs for the mean-field family; other families "
                                      "use SlabKmm (gathered kn)")
        self.model = model
        self.group = group
        if slab is None:
            T = model.toeplitz()
            self._T = T                        # keeps the plan (and its spectrum) alive
            T._plan.trim()                     # the set-up's fp64 transform buffers (GBs at C5)
            slab = SlabToeplitz(T.dims, HipSlabEngine(T._plan), group=group)
        self.slab = slab
        axes = [len(g) for g in model.xgrids]
        if axes[0] <= 1 or len(slab.dims) != sum(1 for m in axes if m > 1):
            raise NotImplementedError("grid-block sharding splits axis 0: it needs more than one point there")

    def elbo_and_grad(self, xbatch, ybatch, noise_std_batch=None, maxiter_cg=10, tol=1e-8, integrated_obs=False,
                      semi_integrated_estimator="analytic", semi_integrated_samps=10, kn_out=None):
        """ELBO (the same on every rank) and theta1 / theta2 .grad set to minus the natural
        gradient, as `MeanFieldToeplitzGP.elbo_and_grad`.  kn_out: a list that receives this
        rank's kn slab and its first expanded-grid column (tests)."""
        from hipgp_amd.dist import allreduce_stats, shared_mc_offset
        m, S = self.model, self.slab
        u = None
        if integrated_obs and semi_integrated_estimator == "mc-biased":
            u = shared_mc_offset(m.kernel.dtype, xbatch.device, self.group)
        a, b = S.my_rows("m")
        Knm, Knn_diag = m._make_grams(xbatch, integrated_obs=integrated_obs,
                                      semi_integrated_estimator=semi_integrated_estimator,
                                      semi_integrated_samps=semi_integrated_samps, mc_offset=u, grid_rows=(a, b))
        with torch.no_grad():
            kn = S.compute_kn(Knm.detach().contiguous(), maxiter=maxiter_cg, tol=tol)
        j0 = S.my_rows("n")[0] * S.rest_n
        if kn_out is not None:
            kn_out.extend([kn, j0])
        stats = m.batch_stats_slab(kn, j0, ybatch, Knn_diag, noise_std_batch,
                                   reduce=lambda t: _allreduce(t, self.group), lead=S.rank == 0)
        del kn
        stats = allreduce_stats(stats, group=self.group)
        return m.apply_stats(stats, xbatch.shape[0])
