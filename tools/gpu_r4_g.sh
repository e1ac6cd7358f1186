# round 4 GPU call G: axes beyond 8192 points (full-grid route for every operator), then the suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_long_axis_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_long_g.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_long_g.log | head -60; [ $rc -le 1 ] || exit 1
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_long_axis_gpu.py > gpurun_out/pytest_gpu_g.log 2>&1
rc=$?; grep -E "FAIL|passed|failed" gpurun_out/pytest_gpu_g.log | tail -10; [ $rc -le 1 ] || exit 1
