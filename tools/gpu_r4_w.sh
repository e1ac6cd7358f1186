# round 4 GPU call W: fp64 operator errors against the oracle on long axes and full-size grids
# (how far from an exact fp64 implementation, after the set-up packing fix).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_long_axis_gpu.py -k "test_beyond_8192_points" -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_w.log 2>&1
rc=$?; grep -E "op err|passed|failed" gpurun_out/pytest_w.log | tail -40; exit $rc
