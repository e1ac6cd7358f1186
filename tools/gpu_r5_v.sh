# round 5 GPU call V: one row pair per 4096-point row-inverse block as the default: the GPU suite,
# C4 K / C^-1 op times, compute_kn phases.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r5v_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5v_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r5v_pytest_gpu.log
for op in K CINV; do
  timeout -k 10 180 python tools/passtime.py --dims 4096,4096 --rhs 25 --op $op 2>/dev/null || exit 1
done | tee gpurun_out/r5v_passtime.txt
timeout -k 10 600 python tools/kn_phases.py --only C2,C3,C4,C5 2>/dev/null | tee gpurun_out/r5v_kn_phases.txt
