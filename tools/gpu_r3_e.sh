# round 3 GPU call E: GPU tests; the driver's bench line; rocprofv3 kernel stats of the bench;
# per-config kernel stats + HBM bytes (C4 K, C3 K, C5 R^T); the five-config coverage bench;
# the C3 minibatch step.  Results under gpurun_out/ (summaries copied to profiles/ afterwards).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_e.log 2>&1; rc=$?
tail -12 gpurun_out/pytest_gpu_e.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || { tail -5 gpurun_out/r3_bench.err; exit 1; }
cat gpurun_out/r3_bench.json
rm -rf gpurun_out/r3_bench_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_bench_prof -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_prof.log 2>&1 || { tail -5 gpurun_out/r3_bench_prof.log; exit 1; }
SHAPE=4096,4096 RHS=25 TAG=C4 timeout -k 10 600 bash tools/prof_cfg.sh || exit 1
SHAPE=2048,2048 RHS=32 TAG=C3 timeout -k 10 600 bash tools/prof_cfg.sh || exit 1
SHAPE=256,256,128 RHS=25 TAG=C5RT OP=RT NOPS=3 timeout -k 10 600 bash tools/prof_cfg.sh || exit 1
timeout -k 10 900 python tools/bench_configs.py > gpurun_out/r3_configs.jsonl 2> gpurun_out/r3_configs.err || { tail -5 gpurun_out/r3_configs.err; exit 1; }
timeout -k 10 400 python tools/c3_step.py 2>&1 | tee gpurun_out/r3_c3_step.jsonl || exit 1
exit $rc
