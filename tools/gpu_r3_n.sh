# round 3 GPU call N: the tree with the PCG epilogue staging and the device-sized 3-D workspace
# budget: GPU tests, smoke, bench line, compute_kn phases, C5 R^T passes, configs table.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_n.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_n.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_n.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_n.log 2>&1 || { tail -20 gpurun_out/smoke_n.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_n.json 2> gpurun_out/bench_n.err || { tail -20 gpurun_out/bench_n.err; exit 1; }
tail -1 gpurun_out/bench_n.json
timeout -k 10 600 python tools/kn_phases.py --only C5,C4,C3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/kn_phases_n.jsonl || exit 1
for op in RT K; do
  timeout -k 10 120 python tools/passtime.py --dims 256,256,128 --rhs 25 --op $op || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/c5_passtime_n.txt || exit 1
timeout -k 10 900 python tools/bench_configs.py > gpurun_out/configs_n.jsonl 2> gpurun_out/configs_n.err || { tail -5 gpurun_out/configs_n.err; exit 1; }
