"""The built libhipgp.so carries no unprotected VMEM store-data hazard: no buffer store of more
than 8 bytes with an SGPR soffset is directly followed by a VALU write of its data VGPRs (the
cause of the round-2 fp64 contiguous-line race).  Static: disassembles the gfx950
code objects, no GPU."""
import os
import shutil

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hipgp_amd", "libhipgp.so")


@pytest.mark.skipif(not (os.path.exists(LIB) and shutil.which("objcopy")
                         and os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump")),
                    reason="needs the built library and the ROCm llvm tools")
def test_no_store_data_hazard():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from hazard_lint import lint, scan
    hits, nstores = lint(LIB)
    assert nstores > 100, nstores           # the scan did see the library's buffer stores
    assert hits == [], hits[:5]
    # the scanner itself: the round-2 pattern is flagged, the protected form is not
    bad = ["  buffer_store_dwordx4 v[96:99], v118, s[8:11], s2 offen", "  v_mul_f64 v[96:97], v[52:53], v[48:49]"]
    good = ["  buffer_store_dwordx4 v[96:99], v118, s[8:11], 0 offen", "  s_nop 0", "  v_mul_f64 v[96:97], v[52:53], v[48:49]"]
    assert len(scan(bad)) == 1 and scan(good) == []
