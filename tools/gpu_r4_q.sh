# round 4 GPU call Q: magnitude-balanced K + i C^-1 set-up packing -- the clamped-case divergence
# diagnostic again, then the whole GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in G4b G7 G4c; do
  echo "== $c"; timeout -k 10 120 python tools/clamp_diag.py $c f64 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/clamp_diag_q.txt || exit 1
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k "solves" -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_q_solves.log 2>&1
grep -E "err vs reference|passed|failed" gpurun_out/pytest_q_solves.log | tail -30
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_q.log 2>&1 || { tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -2 gpurun_out/pytest_q.log
