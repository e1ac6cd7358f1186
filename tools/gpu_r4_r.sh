# round 4 GPU call R: fp64 ops held to 50x the NumPy oracle's own error vs the reference.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k "ops_vs_golden" -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_r.log 2>&1
rc=$?; grep -E " gpu |passed|failed|Error" gpurun_out/pytest_r.log | tail -60; exit $rc
