# round 5 GPU call S: radix-8 tri stages only from 6144 points (C3's 3072-point conv back to
# radix-4): the GPU suite, R^T op times at C2-C4, compute_kn phases.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r5s_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5s_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r5s_pytest_gpu.log
for cfg in "1024,1024 32 RT" "2048,2048 200 RT" "2048,2048 200 R" "4096,4096 25 RT"; do
  set -- $cfg
  timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op $3 2>/dev/null || exit 1
done | tee gpurun_out/r5s_passtime.txt
timeout -k 10 600 python tools/kn_phases.py --only C2,C3,C4 2>/dev/null | tee gpurun_out/r5s_kn_phases.txt
