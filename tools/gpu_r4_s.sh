# round 4 GPU call S: magnitude-balanced gradient cross-correlation (x + i g packing) -- the
# mismatched-scale column-gradient test, then the whole GPU suite and the smoke on this build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_grad_gpu.py -k "mismatched" -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_s_grad.log 2>&1
rc=$?; grep -E "^(K|Cinv|RT|R) |passed|failed" gpurun_out/pytest_s_grad.log | tail -12; [ $rc -eq 0 ] || exit 1
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_s.log 2>&1 || { tail -30 gpurun_out/pytest_s.log; exit 1; }
tail -1 gpurun_out/pytest_s.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s.log 2>&1 || { tail -20 gpurun_out/smoke_s.log; exit 1; }
tail -2 gpurun_out/smoke_s.log
