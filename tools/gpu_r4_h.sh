# round 4 GPU call H: axes beyond 8192 points after the DCT fix
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_long_axis_gpu.py -v --timeout 300 --timeout-method thread -k "beyond or refusals" -s > gpurun_out/pytest_long_h.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert|iterations" gpurun_out/pytest_long_h.log | head -60; [ $rc -le 1 ] || exit 1
