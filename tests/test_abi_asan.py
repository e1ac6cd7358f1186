"""Host-side sanitizer run of the C ABI: tools/asan builds libhipgp's host code with
-fsanitize=address,undefined (device code unchanged, no GPU needed) and runs abi_host_test, which
drives every entry point's argument / state checks, the block geometry and the thread-local error
messages.  Built on first use (about 2 minutes), incremental afterwards."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "tools", "asan")


@pytest.mark.skipif(shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs make + hipcc")
def test_abi_host_sanitizers():
    r = subprocess.run(["make", "-C", ASAN, "-j8", "run"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "all host-side checks passed" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
