# round 5 GPU call X: two row pairs per 2048-point row-inverse block as the default: the GPU suite,
# the five-config table, compute_kn phases, per-pass times of K / R^T at C2-C4, the bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r5x_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5x_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r5x_pytest_gpu.log
timeout -k 10 900 python tools/bench_configs.py > gpurun_out/r5x_configs.jsonl 2> gpurun_out/r5x_configs.err || { tail -5 gpurun_out/r5x_configs.err; exit 1; }
timeout -k 10 600 python tools/kn_phases.py --only C2,C3,C4,C5 2>/dev/null | tee gpurun_out/r5x_kn_phases.jsonl || exit 1
for cfg in "1024,1024 32 K" "2048,2048 200 K" "4096,4096 25 K" "1024,1024 32 RT" "2048,2048 200 RT" "4096,4096 25 RT" "256,256,128 25 K" "256,256,128 25 RT"; do
  set -- $cfg
  timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op $3 2>/dev/null || exit 1
done | tee gpurun_out/r5x_passtime.txt
timeout -k 10 400 python bench.py > gpurun_out/r5x_bench.json 2> gpurun_out/r5x_bench.err || { tail -20 gpurun_out/r5x_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r5x_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['pcg_wall_clock_ms'], d['strong_c4']['ms'])"
