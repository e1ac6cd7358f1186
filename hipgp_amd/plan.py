"""Python handle on one libhipgp plan (one gridded inducing mesh on one device).

Thin: it turns torch tensors into device pointers and calls the C ABI on torch's current
stream.  All arithmetic runs in the HIP kernels of libhipgp.so.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, lib


def expanded_dims(dims):
    """n_i = 2 m_i - 2 (m_i > 1) else m_i  (`hipgp.py:72`)."""
    return tuple(2 * m - 2 if m > 1 else m for m in dims)


# Idle C plans by (dims, dtype, device): the reference builds a fresh ToeplitzTensor on every
# compute_kn call (`hipgp.py:143`); re-using an idle plan of the same grid keeps its twiddle /
# DCT tables and HBM workspaces, so only the spectrum is recomputed (hgp_plan_set_column).
_POOL = {}
_POOL_MAX = 2


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
    def pcg(self, b, maxiter, tol, precond=True, out=None, return_iters=False):
        """Batched PCG with the conj_grad2 recurrence (`cg.py:44-80`), row layout (nrhs, M)."""
        b = self._vec(b, "b", self.M)
        x = torch.empty_like(b) if out is None else out
        self._bind_stream()
        iters = ctypes.c_int(0)
        check(lib().hgp_pcg_solve(self._h, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                  b.shape[0], int(maxiter), float(tol), int(bool(precond)),
                                  _lib.LAYOUT_ROWS, ctypes.byref(iters) if return_iters else None))
        return (x, iters.value) if return_iters else x

    def pcg_steps(self, b, maxiter, tol, precond=True, callback=None):
        """Stepwise PCG for the callback form (`cg.py:77-78`): callback(n, x) after every
        iteration that did not meet the break test; returns x (updated in place)."""
        b = self._vec(b, "b", self.M)
        x = torch.empty_like(b)
        self._bind_stream()
        check(lib().hgp_pcg_begin(self._h, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                  b.shape[0], int(bool(precond)), _lib.LAYOUT_ROWS))
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
        (x, iterations)."""
        import torch.distributed as dist
        b = self._vec(b, "b", self.M)
        x = torch.empty_like(b)
        self._bind_stream()
        check(lib().hgp_pcg_begin(self._h, ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                  b.shape[0], int(bool(precond)), _lib.LAYOUT_ROWS))
        rn = torch.empty(b.shape[0], dtype=self.dtype, device=self.device)
        # the flag travels on the device for RCCL ("nccl"), on the host for gloo
        fdev = "cpu" if dist.get_backend(group) == "gloo" else self.device
        flag = torch.empty(1, dtype=torch.int32, device=fdev)
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
                    idle.append(h)          # stream-ordered re-use (see _POOL)
                else:
                    lib().hgp_plan_destroy(h)
            except Exception:
                pass


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
