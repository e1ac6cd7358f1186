"""Drop-in `ziggy` overlay (SURVEY §8(b) level 1).

Put this repository ahead of a reference checkout on PYTHONPATH and the reference's
experiment scripts run unchanged: the hot-path modules below resolve to the MI355X
implementation in `hipgp_amd.ziggy` (the same module objects, not copies), and every other
`ziggy.*` module (`svgp`, `viz`, `misc.util`, `misc.stats`, `misc.experiment_util`, ...)
resolves to the next `ziggy` package on sys.path (the user's reference checkout), through
the extended package __path__.

  ziggy.hipgp                    -> hipgp_amd.ziggy.hipgp        (`ziggy/hipgp.py`)
  ziggy.kernels                  -> hipgp_amd.ziggy.kernels      (`ziggy/kernels.py`)
  ziggy.svi_gp                   -> hipgp_amd.ziggy.svi_gp       (`ziggy/svi_gp.py`)
  ziggy.misc.toeplitz_tensor     -> hipgp_amd.ziggy.misc.toeplitz_tensor
  ziggy.misc.toeplitz_expanded   -> hipgp_amd.ziggy.misc.toeplitz_expanded
  ziggy.misc.cg                  -> hipgp_amd.ziggy.misc.cg
  ziggy.misc._inv_matmul         -> hipgp_amd.ziggy.misc._inv_matmul
"""
import importlib
import importlib.abc
import importlib.util
import sys
from pkgutil import extend_path

__path__ = extend_path(__path__, __name__)

OVERLAY = {
    "ziggy.hipgp": "hipgp_amd.ziggy.hipgp",
    "ziggy.kernels": "hipgp_amd.ziggy.kernels",
    "ziggy.svi_gp": "hipgp_amd.ziggy.svi_gp",
    "ziggy.misc.toeplitz_tensor": "hipgp_amd.ziggy.misc.toeplitz_tensor",
    "ziggy.misc.toeplitz_expanded": "hipgp_amd.ziggy.misc.toeplitz_expanded",
    "ziggy.misc.cg": "hipgp_amd.ziggy.misc.cg",
    "ziggy.misc._inv_matmul": "hipgp_amd.ziggy.misc._inv_matmul",
}


class _OverlayFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    """Resolves the OVERLAY names to the implementation modules themselves.

    The import system sets `module.__spec__` to the alias's spec after `create_module`
    (`importlib._bootstrap._init_module_attrs`); `exec_module` puts the implementation's own
    spec back, so `__spec__.name == __name__` holds and `importlib.reload` re-executes the
    implementation module."""

    def find_spec(self, fullname, path=None, target=None):
        if fullname in OVERLAY:
            return importlib.util.spec_from_loader(fullname, self)
        return None

    def create_module(self, spec):
        mod = importlib.import_module(OVERLAY[spec.name])
        mod.__dict__.setdefault("_overlay_spec", mod.__spec__)
        return mod

    def exec_module(self, module):
        module.__spec__ = module.__dict__["_overlay_spec"]


if not any(isinstance(f, _OverlayFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _OverlayFinder())
