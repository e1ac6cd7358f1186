"""Dense point-observation cross covariance on the inducing grid via hgp_kuf_grid.

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


def kernel_kind(kernel):
    """HGP_KERN_* code of a ziggy kernel object, or None when the fused kernel does not apply."""
    from hipgp_amd.ziggy import kernels as zk
    if isinstance(kernel, zk.SqExp):
        return _lib.KERN_SQEXP
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
