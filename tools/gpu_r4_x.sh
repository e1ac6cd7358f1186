# round 4 GPU call X: the whole GPU suite and the smoke on the final tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_x.log 2>&1 || { tail -30 gpurun_out/pytest_x.log; exit 1; }
tail -1 gpurun_out/pytest_x.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_x.log 2>&1 || { tail -20 gpurun_out/smoke_x.log; exit 1; }
tail -2 gpurun_out/smoke_x.log
