"""Python handle on one libhipgp plan (one gridded inducing mesh on one device).

Thin: it turns torch tensors into device pointers and calls the C ABI on torch's current
stream.  All arithmetic runs in the HIP kernels of libhipgp.so.
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import check, lib


def expanded_dims(dims):
    """n_i = 2 m_i - 2 (m_i > 1) else m_i  (`hipgp.py:72`)."""
    return tuple(2 * m - 2 if m > 1 else m for m in dims)


# Idle C plans by (dims, dtype, device): the reference builds a fresh ToeplitzTensor on every
# compute_kn call (`hipgp.py:143`); re-using an idle plan of the same grid keeps its twiddle /
# DCT tables, so only the spectrum is recomputed (hgp_plan_set_column).  Idle plans also keep
# their scratch (workspaces, CG vectors: the next solve needs the same sizes) while all idle
# scratch on a device stays under HGP_POOL_MB (default: a quarter of the device's memory, 72 GB
# of the 288 GB: one C5 plan's R^T workspace is 26 GB, and config 4's 200-RHS solve holds 35 GB
# of CG vectors and workspaces -- re-allocating those per compute_kn costs more than it saves;
# with an eighth, round 5's C4 plan (62 GB then, before the fused PCG stopped allocating Ap / z)
# was trimmed after every call); beyond that a plan is trimmed to its tables when it
# goes idle (hgp_plan_trim).
# release_pool() frees every idle plan, e.g. before a large torch allocation (this memory is
# outside torch's caching allocator).
_POOL = {}
_POOL_MAX = 2
_POOL_ENV = os.environ.get("HGP_POOL_MB")
_POOL_DEV = {}
_WS_WARN_BYTES = 4 << 30
_ws_warned = False


def pool_budget(device_index):
    """Idle-plan scratch cap of one device in bytes (HGP_POOL_MB, else 1/4 of its memory)."""
    if _POOL_ENV is not None:
        return int(_POOL_ENV) << 20
    b = _POOL_DEV.get(device_index)
    if b is None:
        b = _POOL_DEV[device_index] = torch.cuda.get_device_properties(device_index).total_memory // 4
    return b


def _scratch_bytes(h):
    b = ctypes.c_int64(0)
    lib().hgp_plan_mem(h, ctypes.byref(b), None)
    return b.value


def pool_scratch_bytes(device_index=None):
    """Device bytes of scratch held by idle pooled plans (of one device, or all)."""
    return sum(_scratch_bytes(h) for k, hs in _POOL.items() for h in hs
               if device_index is None or k[2] == device_index)


def release_pool():
    """Destroy every idle pooled plan (their device memory is outside torch's allocator)."""
    for hs in _POOL.values():
        for h in hs:
            lib().hgp_plan_destroy(h)
    _POOL.clear()


class ToeplitzPlan:
    """Spectra + workspaces for the BTTB operators of one grid (`toeplitz_tensor.py:9-45`)."""

    def __init__(self, dims, dtype=torch.float32, device=None):
        device = torch.device("cuda") if device is None else torch.device(device)
        if device.type != "cuda":
            raise _lib.HipgpError(f"ToeplitzPlan needs a GPU device, got {device} (no CPU fallback)")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.dtype = dtype
        self.dims = tuple(int(m) for m in dims)
        self.ndims = expanded_dims(self.dims)
        self.M = int(np.prod(self.dims))
        self.Mprime = int(np.prod(self.ndims))
        self._key = (self.dims, dtype, device.index)
        idle = _POOL.get(self._key)
        if idle:
            h = idle.pop()
            check(lib().hgp_plan_set_stream(h, _lib.stream_ptr(device)))
        else:
            m = (ctypes.c_int64 * len(self.dims))(*self.dims)
            h = ctypes.c_void_p()
            check(lib().hgp_plan_create(device.index, len(self.dims), m, _lib.dtype_code(dtype), 0,
                                        _lib.stream_ptr(device), ctypes.byref(h)))
        self._h = h
        LK = (ctypes.c_int64 * 3)()
        LR = (ctypes.c_int64 * 3)()
        check(lib().hgp_plan_info(h, None, None, LK, LR))
        self.L_K = tuple(LK)
        self.L_R = tuple(LR)
        self.n_clamped = None

    # -- plumbing --------------------------------------------------------------------------
    def _bind_stream(self):
        check(lib().hgp_plan_set_stream(self._h, _lib.stream_ptr(self.device)))

    def _vec(self, t, name, ncols):
        _lib.require_device_tensor(t, name)
        if t.dtype != self.dtype:
            raise TypeError(f"{name} has dtype {t.dtype}, plan dtype is {self.dtype}")
        if t.device != self.device:
            raise ValueError(f"{name} is on {t.device}, plan on {self.device}")
        if t.dim() != 2 or t.shape[1] != ncols:
            raise ValueError(f"{name} must be (nrhs, {ncols}), got {tuple(t.shape)}")
        return t.contiguous()

    def mem(self):
        """{"scratch": bytes, "tables": bytes} the plan holds outside torch's allocator
        (hgp_plan_mem): workspaces + CG vectors, and spectra + twiddle tables."""
        sb, tb = ctypes.c_int64(0), ctypes.c_int64(0)
        check(lib().hgp_plan_mem(self._h, ctypes.byref(sb), ctypes.byref(tb)))
        return {"scratch": sb.value, "tables": tb.value}

    def trim(self):
        """Free the plan's scratch (workspaces, CG vectors, the set-up transforms' buffers) and keep
        its tables and spectra (hgp_plan_trim); scratch is re-allocated on demand."""
        check(lib().hgp_plan_trim(self._h))

    def _report_ws(self):
        """The first time in a process that a plan's scratch passes 4 GiB, say so once: the 3-D
        operators size their workspace from the device memory (an eighth, at most 32 GiB, so the
        axis-0 spectrum is read once per chunk of many RHS), which a process sharing the GPU
        should know about (HGP_WS_MB caps it; release_pool() frees idle plans)."""
        global _ws_warned
        if _ws_warned:
            return
        sb = _scratch_bytes(self._h)
        if sb > _WS_WARN_BYTES:
            _ws_warned = True
            import warnings
            warnings.warn(f"hipgp plan {self.dims} holds {sb / 2**30:.1f} GiB of device scratch outside torch's "
                          "allocator (workspace budget: HGP_WS_MB; idle plans: hipgp_amd.plan.release_pool())",
                          ResourceWarning, stacklevel=3)

    # -- spectrum ----------------------------------------------------------------------------
    def set_column(self, column, jitter=0.0, clamp_min=1e-6, count_clamped=False):
        """column: kernel-evaluated first row k(x0, x_j), (M,) on the plan device."""
        _lib.require_device_tensor(column, "column")
        col = column.detach().reshape(-1).to(self.dtype).contiguous()
        if col.numel() != self.M:
            raise ValueError(f"column has {col.numel()} values, grid has M={self.M}")
        self._bind_stream()
        n = ctypes.c_int64(-1)
        check(lib().hgp_plan_set_column(self._h, ctypes.c_void_p(col.data_ptr()), float(jitter),
                                        float(clamp_min), ctypes.byref(n) if count_clamped else None))
        self._col_keepalive = col
        if count_clamped:
            self.n_clamped = int(n.value)
        return self.n_clamped

    def spectrum(self, which=_lib.SPEC_D):
        """Real clamped spectrum on the expanded grid (shape ndims): D, sqrt(D) or 1/D."""
        self._bind_stream()
        out = torch.empty(self.ndims, dtype=self.dtype, device=self.device)
        check(lib().hgp_get_spectrum(self._h, int(which), ctypes.c_void_p(out.data_ptr())))
        return out

    # -- operators ---------------------------------------------------------------------------
    def apply(self, op, x, out=None):
        nin = self.Mprime if op == _lib.OP_R else self.M
        nout = self.Mprime if op == _lib.OP_RT else self.M
        x = self._vec(x, "x", nin)
        if out is None:
            out = torch.empty((x.shape[0], nout), dtype=self.dtype, device=self.device)
        self._bind_stream()
        check(lib().hgp_toeplitz_apply(self._h, int(op), ctypes.c_void_p(x.data_ptr()),
                                       ctypes.c_void_p(out.data_ptr()), x.shape[0]))
        if not _ws_warned:
            self._report_ws()
        return out

    def column_grad(self, op, x, g):
        """d/dcolumn of sum(g * op(x)) through the operator's spectrum (hgp_plan_column_grad),
        (M,) in the plan dtype; x, g shaped like op's input / output (`toeplitz_tensor.py:20-125`)."""
        nin = self.Mprime if op == _lib.OP_R else self.M
        nout = self.Mprime if op == _lib.OP_RT else self.M
        x = self._vec(x, "x", nin)
        g = self._vec(g, "g", nout)
        if x.shape[0] != g.shape[0]:
            raise ValueError(f"x has {x.shape[0]} rows, g has {g.shape[0]}")
        out = torch.empty(self.M, dtype=self.dtype, device=self.device)
        self._bind_stream()
        check(lib().hgp_plan_column_grad(self._h, int(op), ctypes.c_void_p(x.data_ptr()),
                                         ctypes.c_void_p(g.data_ptr()), x.shape[0],
                                         ctypes.c_void_p(out.data_ptr())))
        return out

    def dqf(self, left, right):
        """sym_toeplitz_derivative_quadratic_form over the flattened grid (`gpt_toeplitz.py:169-209`)
        through the grid's own factorisation (hgp_plan_dqf): left/right (nvec, M) row layout."""
        left = self._vec(left, "left", self.M)
        right = self._vec(right, "right", self.M)
        if left.shape != right.shape:
            raise ValueError(f"left {tuple(left.shape)} / right {tuple(right.shape)}")
        out = torch.empty(self.M, dtype=self.dtype, device=self.device)
        self._bind_stream()
        check(lib().hgp_plan_dqf(self._h, ctypes.c_void_p(left.data_ptr()), ctypes.c_void_p(right.data_ptr()),
                                 left.shape[0], ctypes.c_void_p(out.data_ptr())))
        return out

    # -- PCG ---------------------------------------------------------------------------------
    def _rhs(self, b, layout):
        """b as the solver takes it: (nrhs, M) rows (conj_grad2) or (M, L) columns (conj_grad)."""
        if layout == _lib.LAYOUT_ROWS:
            b = self._vec(b, "b", self.M)
            return b, b.shape[0]
        _lib.require_device_tensor(b, "b")
        if b.dtype != self.dtype or b.device != self.device:
            raise TypeError(f"b is {b.dtype} on {b.device}, plan is {self.dtype} on {self.device}")
        if b.dim() != 2 or b.shape[0] != self.M:
            raise ValueError(f"b must be (M={self.M}, L) in column layout, got {tuple(b.shape)}")
        return b.contiguous(), b.shape[1]

    def pcg(self, b, maxiter, tol, precond=True, out=None, return_iters=False, layout=_lib.LAYOUT_ROWS):
        """Batched PCG: conj_grad2's recurrence (`cg.py:44-80`) on rows b (nrhs, M), or, with
        layout=LAYOUT_COLS, conj_grad's (`cg.py:5-41`) on columns b (M, L) (the library
        transposes on the device)."""
        b, nrhs = self._rhs(b, layout)
        x = torch.empty_like(b) if out is None else out
        self._bind_stream()
        iters = ctypes.c_int(0)
        check(lib().hgp_pcg_solve(self._h, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                  nrhs, int(maxiter), float(tol), int(bool(precond)),
                                  int(layout), ctypes.byref(iters) if return_iters else None))
        if not _ws_warned:
            self._report_ws()
        return (x, iters.value) if return_iters else x

    def pcg_steps(self, b, maxiter, tol, precond=True, callback=None, layout=_lib.LAYOUT_ROWS):
        """Stepwise PCG for the callback form (`cg.py:77-78`): callback(n, x) after every
        iteration that did not meet the break test; returns x (updated in place; in the
        caller's layout after every step)."""
        b, nrhs = self._rhs(b, layout)
        x = torch.empty_like(b)
        self._bind_stream()
        check(lib().hgp_pcg_begin(self._h, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                  nrhs, int(bool(precond)), int(layout)))
        conv = ctypes.c_int(0)
        for n in range(int(maxiter)):
            check(lib().hgp_pcg_step(self._h, float(tol), ctypes.byref(conv)))
            if conv.value:
                break
            if callback is not None:
                callback(n, x)
        return x

    def pcg_allranks(self, b, maxiter, tol, precond=True, group=None):
        """PCG on this rank's right-hand sides with the reference's break rule applied over
        ALL ranks' RHS (`cg.py:69-71`): each step runs without a local break, then one
        all-reduce(MIN) of "every sqrt(r.r) < tol here" decides for everybody.  Returns
        (x, iterations).

        RCCL ("nccl"): the flag never leaves the device -- hgp_pcg_local_flag, an all-reduce on
        the stream order, hgp_pcg_set_done -- so the host queues `maxiter` steps without a
        synchronisation and the steps after the break are no-ops on the device.  gloo (CPU
        tests): the flag goes through the host each iteration.  A rank with no RHS (a short
        last minibatch) joins the same all-reduces (`pcg_idle_rank`)."""
        import torch.distributed as dist
        if b.shape[0] == 0:
            return torch.empty_like(b), pcg_idle_rank(maxiter, self.device, group)
        b = self._vec(b, "b", self.M)
        x = torch.empty_like(b)
        self._bind_stream()
        check(lib().hgp_pcg_begin(self._h, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                  b.shape[0], int(bool(precond)), _lib.LAYOUT_ROWS))
        if dist.get_backend(group) != "gloo":
            flag = torch.empty(1, dtype=torch.int32, device=self.device)
            for _ in range(int(maxiter)):
                check(lib().hgp_pcg_step(self._h, -1.0, None))
                check(lib().hgp_pcg_local_flag(self._h, float(tol), ctypes.c_void_p(flag.data_ptr())))
                dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
                check(lib().hgp_pcg_set_done(self._h, ctypes.c_void_p(flag.data_ptr())))
            it = ctypes.c_int(0)
            check(lib().hgp_pcg_iters(self._h, ctypes.byref(it)))
            return x, it.value
        rn = torch.empty(b.shape[0], dtype=self.dtype, device=self.device)
        flag = torch.empty(1, dtype=torch.int32)
        it = 0
        for it in range(1, int(maxiter) + 1):
            check(lib().hgp_pcg_step(self._h, -1.0, None))
            check(lib().hgp_pcg_rnorm2(self._h, ctypes.c_void_p(rn.data_ptr())))
            flag.fill_(int(bool(torch.all(torch.sqrt(rn) < tol))))
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
            if int(flag.item()):
                break
        return x, it

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            self._h = None
            try:
                idle = _POOL.setdefault(self._key, [])
                if len(idle) < _POOL_MAX:
                    if pool_scratch_bytes(self._key[2]) + _scratch_bytes(h) > pool_budget(self._key[2]):
                        lib().hgp_plan_trim(h)
                    idle.append(h)          # stream-ordered re-use (see _POOL)
                else:
                    lib().hgp_plan_destroy(h)
            except Exception:
                pass


def pcg_idle_rank(maxiter, device, group=None):
    """The all-reduces of `ToeplitzPlan.pcg_allranks` for a rank that owns no right-hand side:
    it votes "converged" (MIN identity) every iteration and follows the reduced flag, so the
    other ranks never wait on it.  Returns the iteration count the group stopped at."""
    import torch.distributed as dist
    gloo = dist.get_backend(group) == "gloo"
    flag = torch.ones(1, dtype=torch.int32, device="cpu" if gloo else device)
    if gloo:
        it = 0
        for it in range(1, int(maxiter) + 1):
            flag.fill_(1)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
            if int(flag.item()):
                break
        return it
    # RCCL: no host round trip per iteration; count on the device the iterations up to and
    # including the first whose reduced flag is 1 -- the count the active ranks report
    # (hgp_pcg_iters) -- and read it once at the end
    count = torch.zeros(1, dtype=torch.int32, device=device)
    stopped = torch.zeros(1, dtype=torch.int32, device=device)
    for _ in range(int(maxiter)):
        flag.fill_(1)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        count += 1 - stopped
        torch.maximum(stopped, flag, out=stopped)
    return int(count.item())


def sym_toeplitz_dqf(left_vectors, right_vectors):
    """gpytorch's sym_toeplitz_derivative_quadratic_form (`ziggy/misc/gpt_toeplitz.py:169-209`):
    left/right (n,) or (n, s) as the reference takes them; returns (n,) with
    out[i] = sum_j left[:, j]^T (dT/dc_i) right[:, j]  (ones on the i-th sub/super-diagonal)."""
    _lib.require_device_tensor(left_vectors, "left_vectors")
    if left_vectors.ndimension() == 1:
        left_vectors = left_vectors.unsqueeze(1)
        right_vectors = right_vectors.unsqueeze(1)
    if left_vectors.shape != right_vectors.shape or left_vectors.dim() != 2:
        raise ValueError(f"left {tuple(left_vectors.shape)} / right {tuple(right_vectors.shape)}: "
                         "expected matching (n, s)")
    n = left_vectors.shape[0]
    u = left_vectors.t().contiguous()
    v = right_vectors.t().contiguous().to(u.dtype)
    out = torch.empty(n, dtype=u.dtype, device=u.device)
    check(lib().hgp_sym_toeplitz_dqf(_lib.dtype_code(u.dtype), ctypes.c_void_p(u.data_ptr()),
                                     ctypes.c_void_p(v.data_ptr()), u.shape[0], n,
                                     ctypes.c_void_p(out.data_ptr()), _lib.stream_ptr(u.device)))
    return out


def rowdot(a, c):
    """out[b] = sum_j a[b, j] c[b, j] on the device (`cg.py:64` style dots)."""
    _lib.require_device_tensor(a, "a")
    a = a.contiguous()
    c = c.contiguous()
    out = torch.empty(a.shape[0], dtype=a.dtype, device=a.device)
    check(lib().hgp_rowdot(_lib.dtype_code(a.dtype), ctypes.c_void_p(a.data_ptr()),
                           ctypes.c_void_p(c.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                           a.shape[0], a.shape[1], _lib.stream_ptr(a.device)))
    return out
