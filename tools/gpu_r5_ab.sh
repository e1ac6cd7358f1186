# round 5 GPU call AB: radix-8 grouped 12288-point rows as the default: the GPU suite, smoke, R / R^T
# op times at C2-C5, compute_kn phases.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r5ab_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5ab_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r5ab_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5ab_smoke.log 2>&1 || { tail -20 gpurun_out/r5ab_smoke.log; exit 1; }
tail -2 gpurun_out/r5ab_smoke.log
for cfg in "4096,4096 25 RT" "4096,4096 25 R" "2048,2048 200 RT" "1024,1024 32 RT"; do
  set -- $cfg
  timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op $3 2>/dev/null || exit 1
done | tee gpurun_out/r5ab_passtime.txt
timeout -k 10 600 python tools/kn_phases.py --only C2,C3,C4,C5 2>/dev/null | tee gpurun_out/r5ab_kn_phases.txt
