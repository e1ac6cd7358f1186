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


def _a2a(out, inp, out_splits, in_splits, group):
    """all_to_all_single on real views (complex / CUDA through the host for gloo)."""
    gloo = dist.get_backend(group) == "gloo"
    i = torch.view_as_real(inp).reshape(-1) if inp.is_complex() else inp.reshape(-1)
    o = torch.view_as_real(out).reshape(-1) if out.is_complex() else out.reshape(-1)
    f = 2 if inp.is_complex() else 1
    if gloo and i.is_cuda:
        ih, oh = i.cpu(), torch.empty(o.shape, dtype=o.dtype)
        dist.all_to_all_single(oh, ih, [f * s for s in out_splits], [f * s for s in in_splits], group=group)
        o.copy_(oh)
    else:
        dist.all_to_all_single(o, i, [f * s for s in out_splits], [f * s for s in in_splits], group=group)
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
    """The slab stages on libhipgp (hgp_slab_pass), one replicated plan per rank."""

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

    def _run(self, op, stage, x, y, nrhs, nrows, g0=0, ng=0):
        self.plan._bind_stream()
        check(lib().hgp_slab_pass(self.plan._h, int(op), int(stage), ctypes.c_void_p(x.data_ptr()),
                                  ctypes.c_void_p(y.data_ptr()), nrhs, nrows, g0, ng))

    def fwd(self, op, x, nrows, E):
        self._run(op, _lib.SLAB_FWD, x.contiguous(), E, x.shape[0], nrows)

    def conv(self, op, lines, g0, ng, nrhs):
        self._run(op, _lib.SLAB_CONV, lines, lines, nrhs, 0, g0, ng)

    def conv_a2a(self, op, recv, send, g0, ng, nrhs, ws):
        self._run(op, _lib.SLAB_CONV_A2A, recv, send, nrhs, ws, g0, ng)

    def inv(self, op, E, nrows, y):
        self._run(op, _lib.SLAB_INV, E, y, y.shape[0], nrows)


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
    def apply(self, op, x):
        """op (libhipgp OP_*) on this rank's slab x (nrhs, local in-size) -> local out slab."""
        e = self.engine
        ws, rk = self.ws, self.rank
        rows_in = self.rows_n if op == _lib.OP_R else self.rows_m
        rows_out = self.rows_n if op == _lib.OP_RT else self.rows_m
        rest_out = self.rest_n if op == _lib.OP_RT else self.rest_m
        in0 = self.ndims[0] if op == _lib.OP_R else self.dims[0]
        out0 = self.ndims[0] if op == _lib.OP_RT else self.dims[0]
        P0 = max(in0, out0)
        nrhs = x.shape[0]
        NG, inner = e.geometry(op)
        groups = [split(NG, ws, k) for k in range(ws)]
        gs0, gs1 = groups[rk]
        ng = gs1 - gs0
        ni = rows_in[rk][1] - rows_in[rk][0]
        no = rows_out[rk][1] - rows_out[rk][0]
        cd, dev = e.cdtype, x.device
        # 1. local transforms along the other axes: E[g][q][i][c] over my input rows
        E = torch.empty((NG, nrhs, ni, inner), dtype=cd, device=dev)
        if ni > 0:
            e.fwd(op, x, ni, E)
        # 2. all-to-all: my rows of every group -> all rows of my groups, received as rank blocks
        #    [r][g][q][i - a_r][c] (rank r's rows [a_r, a_r + cnt_r))
        sizes_in = [(groups[s][1] - groups[s][0]) * nrhs * ni * inner for s in range(ws)]
        sizes_rx = [ng * nrhs * (rows_in[r][1] - rows_in[r][0]) * inner for r in range(ws)]
        recv = torch.empty(sum(sizes_rx), dtype=cd, device=dev)
        _a2a(recv, E.reshape(-1), sizes_rx, sizes_in, self.group)
        # 3. the axis-0 convolution on my groups straight from the receive buffer into the send
        #    buffer of the return all-to-all, rank blocks [r][g][q][o - b_r][c] of the output rows
        #    (HGP_SLAB_CONV_A2A: no line buffer, no gather / scatter copies)
        sizes_tx = [ng * nrhs * (rows_out[r][1] - rows_out[r][0]) * inner for r in range(ws)]
        send = torch.empty(sum(sizes_tx), dtype=cd, device=dev)
        if ng > 0:
            e.conv_a2a(op, recv, send, gs0, ng, nrhs, ws)
        # 4. all-to-all back: all rows of my groups -> my output rows of every group
        back = torch.empty(NG * nrhs * no * inner, dtype=cd, device=dev)
        sizes_back = [(groups[s][1] - groups[s][0]) * nrhs * no * inner for s in range(ws)]
        _a2a(back, send, sizes_back, sizes_tx, self.group)
        E2 = back.view(NG, nrhs, no, inner)      # groups arrive in rank order = group order
        # 5. local inverse transforms over my output rows
        y = torch.empty((nrhs, no * rest_out), dtype=x.dtype, device=dev)
        if no > 0:
            e.inv(op, E2, no, y)
        return y

    # -- PCG -------------------------------------------------------------------------------
    def dot(self, a, b):
        """Global per-RHS dot products: local row sums, one all-reduce of nrhs values."""
        s = (a * b).sum(dim=1) if a.shape[1] else a.new_zeros(a.shape[0])
        return _allreduce(s.contiguous(), self.group)

    def pcg(self, b, maxiter=20, tol=1e-8, precond=True, callback=None):
        """conj_grad2 (`cg.py:44-80`) on the slabs: x0 = 0, per-RHS alpha / beta from all-reduced
        dots, break when EVERY global sqrt(r.r) < tol.  Returns (x, iterations run).

        The break is decided on the device: every rank holds the same reduced r.r, so a device
        flag `done` (all sqrt(r.r) < tol after some iteration) is identical everywhere; the
        iterations after it leave x unchanged (alpha masked to 0, the same x as the reference's
        break) and the host queues all `maxiter` iterations without a synchronisation (RCCL: the
        dots' all-reduces are stream-ordered).  The iteration count is read once at the end.
        With a callback (`cg.py:77-78`, called after every iteration that did not break) the
        host must look at the flag, so that form synchronises per iteration as the reference."""
        P = (lambda v: self.apply(_lib.OP_CINV, v)) if precond else (lambda v: v)
        x = torch.zeros_like(b)
        r = b.clone()
        z = P(r)
        p = z
        rs = self.dot(r, z)
        done = torch.zeros((), dtype=torch.bool, device=b.device)
        its = torch.zeros((), dtype=torch.int64, device=b.device)
        for n in range(int(maxiter)):
            its += (~done).long()
            Ap = self.apply(_lib.OP_K, p)
            # after the break every update is masked out (alpha = 0), so x stays the iterate the
            # reference returns; torch.where keeps the 0/0 of the masked iterations out
            alpha = torch.where(done, torch.zeros_like(rs), rs / self.dot(p, Ap))
            x = x + alpha.unsqueeze(-1) * p
            r = r - alpha.unsqueeze(-1) * Ap
            rnew = self.dot(r, r)
            done = done | torch.all(torch.sqrt(rnew) < tol)
            if callback is not None:
                if bool(done):
                    break
            z = P(r)
            zr = self.dot(z, r)
            beta = zr / rs
            # p = 0 once done: the masked iterations then see Ap = 0 and finite x, r
            p = torch.where(done, torch.zeros((), dtype=p.dtype, device=p.device), z + beta.unsqueeze(-1) * p)
            rs = zr                   # = sum(r * z) at the top of the next iteration (cg.py:64)
            if callback is not None:
                callback(n, x)
        return x, int(its)

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
