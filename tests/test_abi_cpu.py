"""CPU-side checks: the C-ABI library loads and exports every symbol include/hipgp.h
declares; argument validation that happens before any HIP call; host-side shape logic.
(No compute calls: there is no GPU in the build container.)"""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "hipgp.h")).read()
    return sorted(set(re.findall(r"\b(hgp_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from hipgp_amd import _lib
    L = _lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(L, s), f"libhipgp.so does not export {s}"
    assert set(syms) == set(_lib.EXPORTS)


def test_version_and_arg_errors_without_gpu():
    from hipgp_amd import _lib
    L = _lib.lib()
    assert b"gfx950" in L.hgp_version()
    h = ctypes.c_void_p()
    m = (ctypes.c_int64 * 1)(8)
    rc = L.hgp_plan_create(0, 0, m, 0, 0, None, ctypes.byref(h))     # ndim=0 rejected before HIP
    assert rc == -1 and b"ndim" in L.hgp_last_error()
    rc = L.hgp_plan_create(0, 1, m, 7, 0, None, ctypes.byref(h))     # bad dtype
    assert rc == -1 and b"dtype" in L.hgp_last_error()
    assert L.hgp_toeplitz_apply(None, 0, None, None, 1) == -1
    assert L.hgp_plan_destroy(None) == 0


def test_expanded_dims_and_fft_lengths():
    from hipgp_amd.plan import expanded_dims
    assert expanded_dims((1024, 1024)) == (2046, 2046)
    assert expanded_dims((37, 3, 1)) == (72, 4, 1)
    # the padded power-of-two lengths the plan uses: L_K >= 2m-1, L_R >= 4m-4
    nxt = lambda v: 1 << (v - 1).bit_length()
    for m in (2, 3, 37, 256, 1024, 4096):
        assert nxt(2 * m - 1) >= 2 * m - 1 and nxt(4 * m - 4) >= (2 * m - 2) + m - 1


def test_cpu_tensors_are_refused():
    """No CPU fallback: the product path raises for CPU tensors."""
    import torch
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    with pytest.raises(_lib.HipgpError):
        ToeplitzPlan((8, 8), torch.float32, torch.device("cpu"))
