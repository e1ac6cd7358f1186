# round 4 GPU call A: the restored tree end to end (GPU tests, smoke, bench, bench kernel stats),
# then evidence for this round's targets: C4 R^T kernel stats + per-kernel PMC bytes against B_RT
# and the L_R floor, C5 R^T the same, and the C4 / C3 K op under larger 2-D workspace budgets
# (fewer spectrum re-reads).  Each GPU step under its own limit; results under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread --ignore=tests/test_fit_c3_gpu.py > gpurun_out/pytest_gpu_a.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_a.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_a.log
# the new G19 tests: an assertion failure (rc 1) does not stop the measurements, a crash does
timeout -k 10 600 python -u -m pytest tests/test_fit_c3_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_c3_a.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_c3_a.log; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_a.log 2>&1 || { tail -20 gpurun_out/smoke_a.log; exit 1; }
tail -2 gpurun_out/smoke_a.log
timeout -k 10 400 python bench.py > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err || { tail -20 gpurun_out/bench_a.err; exit 1; }
tail -1 gpurun_out/bench_a.json
bash tools/profile.sh r4a || exit 1
SHAPE=4096,4096 RHS=25 TAG=C4RT OP=RT NOPS=3 timeout -k 10 600 bash tools/prof_cfg.sh || exit 1
SHAPE=256,256,128 RHS=25 TAG=C5RT OP=RT NOPS=3 timeout -k 10 600 bash tools/prof_cfg.sh || exit 1
for ws in 0 4096 16384; do
  for cfg in "4096,4096 25" "2048,2048 200"; do
    set -- $cfg
    if [ $ws = 0 ]; then
      timeout -k 10 120 python tools/passtime.py --dims $1 --rhs $2 --op K || exit 1
    else
      HGP_WS_MB=$ws timeout -k 10 120 python tools/passtime.py --dims $1 --rhs $2 --op K || exit 1
    fi
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ws2d_a.txt || exit 1
timeout -k 10 900 python tools/c3_step.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/c3_fit_a.jsonl || exit 1
