"""Cross covariances on the inducing grid: point observations (hgp_kuf_grid) and line-integral
observations (hgp_kuf_semi_mc / hgp_kuf_semi_sqexp / hgp_knn_doubly_diag).

`svi_gp._make_grams` (`svi_gp.py:48-76`) evaluates Knm = kernel(xbatch, xinduce) through the
(B, M, D) broadcast of `kernels.py:78,149`; this computes the same values with one fused HIP
kernel straight into the (B, M) layout the PCG reads.  Used when the kernel is SqExp or
Matern(nu in {1/2, 3/2, 5/2}) with a scalar length scale and no gradient is needed; other
kernels (or kernel-hyper-parameter learning) evaluate the torch kernel on the device.
"""
import ctypes

import torch

from . import _lib
from ._lib import check, lib


def kernel_kind(kernel, gneiting=False):
    """HGP_KERN_* code of a ziggy kernel object, or None when the fused kernel does not apply."""
    from hipgp_amd.ziggy import kernels as zk
    if isinstance(kernel, zk.SqExp):
        return _lib.KERN_SQEXP
    if gneiting and isinstance(kernel, zk.Gneiting):
        return _lib.KERN_GNEITING
    if isinstance(kernel, zk.Matern):
        return {0.5: _lib.KERN_MATERN12, 1.5: _lib.KERN_MATERN32, 2.5: _lib.KERN_MATERN52}.get(kernel.nu)
    return None


def _scalar(v):
    if torch.is_tensor(v):
        if v.numel() != 1:
            return None
        return float(v.detach().reshape(()).item())
    return float(v)


def kuf_grid(kernel, xgrids, x, params):
    """Knm (nobs, M) for observations x (nobs, D) against the C-order mesh of xgrids, or None
    when the fused path does not apply (caller then evaluates the torch kernel)."""
    kind = kernel_kind(kernel)
    if kind is None or x.device.type != "cuda" or x.dim() != 2 or x.shape[1] != len(xgrids):
        return None
    if x.dtype not in (torch.float32, torch.float64) or len(xgrids) > 3:
        return None
    sig2, ell = params
    if torch.is_grad_enabled() and any(torch.is_tensor(p) and p.requires_grad for p in (sig2, ell, x)):
        return None
    s2, el = _scalar(sig2), _scalar(ell)
    if s2 is None or el is None:
        return None
    grids = [g.to(device=x.device, dtype=x.dtype).contiguous() for g in xgrids]
    xc = x.detach().contiguous()
    M = 1
    for g in grids:
        M *= g.numel()
    out = torch.empty((x.shape[0], M), dtype=x.dtype, device=x.device)
    m = (ctypes.c_int64 * len(grids))(*[g.numel() for g in grids])
    ptrs = (ctypes.c_void_p * len(grids))(*[g.data_ptr() for g in grids])
    check(lib().hgp_kuf_grid(_lib.dtype_code(x.dtype), kind, len(grids), m, ptrs, ctypes.c_void_p(xc.data_ptr()),
                             x.shape[0], s2, el, ctypes.c_void_p(out.data_ptr()), _lib.stream_ptr(x.device)))
    return out


def _grid_call_args(kernel, xgrids, x, params, gneiting=False):
    """(kind, s2, el, grids, xc, M) for the fused grid kernels, or None when they do not apply."""
    kind = kernel_kind(kernel, gneiting=gneiting)
    if kind is None or x.device.type != "cuda" or x.dim() != 2 or x.shape[1] != len(xgrids):
        return None
    if x.dtype not in (torch.float32, torch.float64) or len(xgrids) > 3:
        return None
    sig2, ell = params
    if torch.is_grad_enabled() and any(torch.is_tensor(p) and p.requires_grad for p in (sig2, ell, x)):
        return None
    s2, el = _scalar(sig2), _scalar(ell)
    if s2 is None or el is None:
        return None
    grids = [g.to(device=x.device, dtype=x.dtype).contiguous() for g in xgrids]
    M = 1
    for g in grids:
        M *= g.numel()
    return kind, s2, el, grids, x.detach().contiguous(), M


def _grid_ptrs(grids):
    m = (ctypes.c_int64 * len(grids))(*[g.numel() for g in grids])
    ptrs = (ctypes.c_void_p * len(grids))(*[g.data_ptr() for g in grids])
    return m, ptrs


def kuf_semi_mc(kernel, xgrids, x, params, npts, u=None):
    """Line-integral Knm (nobs, M) by the reference's biased Monte-Carlo estimator
    (`Kernel.k_semi_mc` `kernels.py:19-39`, as `svi_gp.py:61-64` uses it), or None when the
    fused path does not apply.  Consumes one torch.rand(1) draw exactly as the reference, or
    uses the given offset draw `u` (a 1-element tensor in [0, 1))."""
    a = _grid_call_args(kernel, xgrids, x, params, gneiting=True)
    if a is None:
        return None
    kind, s2, el, grids, xc, M = a
    if u is None:
        u = torch.rand(1, dtype=kernel.dtype, device=x.device)          # kernels.py:28-29
    u = u.to(device=x.device, dtype=x.dtype).reshape(1).contiguous()
    out = torch.empty((x.shape[0], M), dtype=x.dtype, device=x.device)
    m, ptrs = _grid_ptrs(grids)
    kp = float(getattr(kernel, "alpha", 1.))
    check(lib().hgp_kuf_semi_mc(_lib.dtype_code(x.dtype), kind, kp, len(grids), m, ptrs,
                                ctypes.c_void_p(xc.data_ptr()), x.shape[0], s2, el, int(npts),
                                ctypes.c_void_p(u.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                _lib.stream_ptr(x.device)))
    return out


def kuf_semi_sqexp(kernel, xgrids, x, params):
    """Analytic SqExp line-integral Knm (nobs, M) (`SqExp.k_semi` `kernels.py:80-85` ->
    `semi_integrated_sqe` `:223-237`), or None when the fused path does not apply."""
    a = _grid_call_args(kernel, xgrids, x, params)
    if a is None or a[0] != _lib.KERN_SQEXP:
        return None
    kind, s2, el, grids, xc, M = a
    out = torch.empty((x.shape[0], M), dtype=x.dtype, device=x.device)
    m, ptrs = _grid_ptrs(grids)
    check(lib().hgp_kuf_semi_sqexp(_lib.dtype_code(x.dtype), len(grids), m, ptrs, ctypes.c_void_p(xc.data_ptr()),
                                   x.shape[0], s2, el, ctypes.c_void_p(out.data_ptr()), _lib.stream_ptr(x.device)))
    return out


def knn_doubly_diag(table, x, params):
    """Knn_diag (nobs,) of line-integral observations by the reference's table interpolation
    (`KernelDoublyDiagInterpolator.forward` `kernels.py:200-220`); table: device tensor (3, N)
    = distance grid, knn, slopes in x.dtype."""
    _lib.require_device_tensor(x, "x")
    sig2, ell = params
    s2, el = _scalar(sig2), _scalar(ell)
    if s2 is None or el is None:
        raise _lib.HipgpError("k_doubly_diag: sig2 / ell must be scalars")
    xc = x.detach().contiguous()
    tab = table.to(device=x.device, dtype=x.dtype).contiguous()
    out = torch.empty((x.shape[0],), dtype=x.dtype, device=x.device)
    check(lib().hgp_knn_doubly_diag(_lib.dtype_code(x.dtype), x.shape[1], ctypes.c_void_p(xc.data_ptr()), x.shape[0],
                                    s2, el, ctypes.c_void_p(tab.data_ptr()), tab.shape[1],
                                    ctypes.c_void_p(out.data_ptr()), _lib.stream_ptr(x.device)))
    return out
