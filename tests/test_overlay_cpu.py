"""The `ziggy` drop-in overlay (SURVEY §8(b) level 1): with this repository ahead of a
reference checkout on PYTHONPATH, the reference's experiment modules import, the hot-path
modules are this repo's (the same module objects as hipgp_amd.ziggy), and every other
`ziggy.*` module is the reference's.  Runs in a subprocess so the overlay's package path is
computed from that PYTHONPATH.  No GPU, no compute."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

PROBE = r"""
import sys, types
sys.dont_write_bytecode = True
# seaborn (plot styling) is not installed in this image; the modules only call set_style
sys.modules.setdefault("seaborn", types.SimpleNamespace(set_style=lambda *a, **k: None))
import ziggy.misc.experiment_util as eu
import ziggy.hipgp, ziggy.kernels, ziggy.svi_gp, ziggy.svgp, ziggy.misc.util, ziggy.misc.stats
import ziggy.misc.toeplitz_tensor, ziggy.misc.toeplitz_expanded, ziggy.misc.cg, ziggy.misc._inv_matmul
import hipgp_amd.ziggy.hipgp as H, hipgp_amd.ziggy.misc.toeplitz_tensor as T, hipgp_amd.ziggy.svi_gp as S
assert ziggy.misc.toeplitz_tensor is T and ziggy.hipgp is H and ziggy.svi_gp is S
assert eu.hipgp is H, eu.hipgp
assert ziggy.svgp.SviGP is S.SviGP          # the reference SVGP baseline runs on our driver
for m in (ziggy.svgp, ziggy.misc.util, ziggy.misc.stats, eu):
    assert m.__file__.startswith(sys.argv[1]), m.__file__
for m in (ziggy.hipgp, ziggy.kernels, ziggy.misc.toeplitz_expanded, ziggy.misc.cg, ziggy.misc._inv_matmul):
    assert m.__file__.startswith(sys.argv[2]), m.__file__
assert callable(H.MeanFieldToeplitzGP.fit) and callable(H.MeanFieldToeplitzGP.batch_solve)
print("overlay ok")
"""


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "ziggy")), reason="no reference checkout here")
def test_overlay_resolves_reference_modules():
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([ROOT, REF]), PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-c", PROBE, REF, os.path.join(ROOT, "hipgp_amd")], env=env,
                       capture_output=True, text=True, timeout=240, cwd="/tmp")
    assert r.returncode == 0 and "overlay ok" in r.stdout, r.stdout + r.stderr


def test_overlay_without_reference():
    """Alone (the GPU box has no reference), the hot-path modules still import."""
    env = dict(os.environ, PYTHONPATH=ROOT, PYTHONDONTWRITEBYTECODE="1")
    code = ("import importlib, ziggy.hipgp, ziggy.misc.toeplitz_tensor as t, hipgp_amd.ziggy.misc.toeplitz_tensor as u;"
            "import ziggy.misc.cg as c;"
            "assert t is u;"
            "assert all(m.__spec__.name == m.__name__ for m in (t, c, ziggy.hipgp)), [t.__spec__.name, c.__spec__.name];"
            "f = c.conj_grad2; importlib.reload(c); assert c.conj_grad2 is not f;"   # reload re-executes the module
            "importlib.reload(ziggy.misc.cg); assert ziggy.misc.cg is c;"
            "print('alone ok')")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240,
                       cwd="/tmp")
    assert r.returncode == 0 and "alone ok" in r.stdout, r.stdout + r.stderr
