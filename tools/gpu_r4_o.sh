# round 4 GPU call O: the clamped 20-iteration goldens held to the reference's own chaotic spread
# (golden_cases.chaotic_bound), printing each error beside that spread.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k "solves" -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_o.log 2>&1
rc=$?; grep -E "err vs reference|passed|failed|Error" gpurun_out/pytest_o.log | tail -40; exit $rc
