# round 4 GPU call F: G = 4 grouped 4096-point rows by default -- the GPU suite, C4 / C3 phases,
# K / C^-1 / R^T at C4, the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_f.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_f.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_f.log
timeout -k 10 600 python tools/kn_phases.py --only C4,C3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/kn_phases_f.jsonl || exit 1
for op in K CINV RT; do
  timeout -k 10 120 python tools/passtime.py --dims 4096,4096 --rhs 25 --op $op || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/c4_ops_f.txt || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_f.json 2> gpurun_out/bench_f.err || { tail -20 gpurun_out/bench_f.err; exit 1; }
tail -1 gpurun_out/bench_f.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['pcg_wall_clock_ms'], d['roofline']['frac'])"
