"""ctypes binding of libhipgp.so (the C ABI declared in include/hipgp.h).

The library is built in-tree by `__graft_entry__.build()` (hipcc --offload-arch=gfx950).
There is no fallback: if the library is missing or fails to load, every entry point raises.
torch is imported first so that libhipgp.so binds to the HIP runtime torch already loaded
(same SONAME libamdhip64.so.7) — one runtime, one device context per process.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen below, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
# HGP_LIB selects an alternative in-tree build (block-shape variants for tuning runs)
LIB_PATH = os.environ.get("HGP_LIB") or os.path.join(_HERE, "libhipgp.so")

HGP_F32, HGP_F64 = 0, 1
OP_K, OP_CINV, OP_RT, OP_R = 0, 1, 2, 3
SPEC_D, SPEC_DSQRT, SPEC_DI = 0, 1, 2
LAYOUT_ROWS, LAYOUT_COLS = 0, 1
SLAB_FWD, SLAB_CONV, SLAB_INV, SLAB_CONV_A2A = 0, 1, 2, 3

# every symbol include/hipgp.h declares (tests check the library exports all of them)
EXPORTS = (
    "hgp_plan_create", "hgp_plan_set_stream", "hgp_plan_set_column", "hgp_toeplitz_apply",
    "hgp_pcg_solve", "hgp_pcg_begin", "hgp_pcg_step", "hgp_get_spectrum", "hgp_rowdot",
    "hgp_plan_info", "hgp_plan_destroy", "hgp_last_error", "hgp_version",
    "hgp_toeplitz_apply_pass", "hgp_op_pass_count", "hgp_pcg_rnorm2", "hgp_kuf_grid",
    "hgp_kuf_semi_mc", "hgp_kuf_semi_sqexp", "hgp_knn_doubly_diag", "hgp_meanfield_stats",
    "hgp_block_stats", "hgp_sym_toeplitz_dqf", "hgp_plan_column_grad",
    "hgp_plan_dqf", "hgp_pcg_local_flag", "hgp_pcg_set_done", "hgp_pcg_iters",
    "hgp_slab_info", "hgp_slab_pass", "hgp_plan_mem", "hgp_plan_trim",
    "hgp_slab_pass_ex", "hgp_slab_cg_xr", "hgp_slab_cg_check", "hgp_slab_cg_p",
    "hgp_meanfield_rowdots", "hgp_meanfield_cols",
)
KERN_SQEXP, KERN_MATERN12, KERN_MATERN32, KERN_MATERN52, KERN_GNEITING = 0, 1, 2, 3, 4


class HipgpError(RuntimeError):
    pass


_lib = None


def lib():
    """Load (once) and return the ctypes library handle; raise if it is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HipgpError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    vp, i64, i32, dbl = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double
    pi64, pi32 = ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int)
    sig = {
        "hgp_plan_create": (i32, [i32, i32, pi64, i32, i64, vp, ctypes.POINTER(vp)]),
        "hgp_plan_set_stream": (i32, [vp, vp]),
        "hgp_plan_set_column": (i32, [vp, vp, dbl, dbl, pi64]),
        "hgp_toeplitz_apply": (i32, [vp, i32, vp, vp, i64]),
        "hgp_pcg_solve": (i32, [vp, vp, vp, i64, i32, dbl, i32, i32, pi32]),
        "hgp_pcg_begin": (i32, [vp, vp, vp, i64, i32, i32]),
        "hgp_pcg_step": (i32, [vp, dbl, pi32]),
        "hgp_get_spectrum": (i32, [vp, i32, vp]),
        "hgp_rowdot": (i32, [i32, vp, vp, vp, i64, i64, vp]),
        "hgp_plan_info": (i32, [vp, pi64, pi64, pi64, pi64]),
        "hgp_plan_destroy": (i32, [vp]),
        "hgp_last_error": (ctypes.c_char_p, []),
        "hgp_version": (ctypes.c_char_p, []),
        "hgp_toeplitz_apply_pass": (i32, [vp, i32, vp, vp, i64, i32]),
        "hgp_op_pass_count": (i32, [vp]),
        "hgp_pcg_rnorm2": (i32, [vp, vp]),
        "hgp_kuf_grid": (i32, [i32, i32, i32, pi64, ctypes.POINTER(vp), vp, i64, dbl, dbl, vp, vp]),
        "hgp_kuf_semi_mc": (i32, [i32, i32, dbl, i32, pi64, ctypes.POINTER(vp), vp, i64, dbl, dbl, i32, vp, vp, vp]),
        "hgp_kuf_semi_sqexp": (i32, [i32, i32, pi64, ctypes.POINTER(vp), vp, i64, dbl, dbl, vp, vp]),
        "hgp_knn_doubly_diag": (i32, [i32, i32, vp, i64, dbl, dbl, vp, i32, vp, vp]),
        "hgp_meanfield_stats": (i32, [i32, vp, i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "hgp_meanfield_rowdots": (i32, [i32, vp, i64, i64, vp, vp, vp, vp]),
        "hgp_meanfield_cols": (i32, [i32, vp, i64, i64, vp, vp, vp, vp, vp]),
        "hgp_block_stats": (i32, [i32, i32, pi64, pi64, vp, i64, vp, vp, vp, vp, vp, vp]),
        "hgp_sym_toeplitz_dqf": (i32, [i32, vp, vp, i64, i64, vp, vp]),
        "hgp_plan_column_grad": (i32, [vp, i32, vp, vp, i64, vp]),
        "hgp_plan_dqf": (i32, [vp, vp, vp, i64, vp]),
        "hgp_pcg_local_flag": (i32, [vp, dbl, vp]),
        "hgp_pcg_set_done": (i32, [vp, vp]),
        "hgp_pcg_iters": (i32, [vp, pi32]),
        "hgp_slab_info": (i32, [vp, i32, pi64, pi64]),
        "hgp_plan_mem": (i32, [vp, pi64, pi64]),
        "hgp_plan_trim": (i32, [vp]),
        "hgp_slab_pass": (i32, [vp, i32, i32, vp, vp, i64, i64, i64, i64]),
        "hgp_slab_pass_ex": (i32, [vp, i32, i32, vp, vp, i64, i64, i64, i64, vp, vp, vp]),
        "hgp_slab_cg_xr": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, vp]),
        "hgp_slab_cg_check": (i32, [vp, vp, i64, dbl, vp, vp]),
        "hgp_slab_cg_p": (i32, [vp, vp, vp, vp, vp, i64, i64, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc):
    if rc != 0:
        msg = lib().hgp_last_error().decode(errors="replace")
        raise HipgpError(f"libhipgp error {rc}: {msg}")
    return rc


def dtype_code(dtype):
    if dtype == torch.float32:
        return HGP_F32
    if dtype == torch.float64:
        return HGP_F64
    raise TypeError(f"unsupported dtype {dtype} (float32 / float64 only)")


def stream_ptr(device):
    """Raw hipStream_t of torch's current stream on `device`."""
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device_tensor(t, name):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise HipgpError(f"{name} is on {t.device}: the HIP path runs on a GPU device only "
                         "(no CPU fallback)")
