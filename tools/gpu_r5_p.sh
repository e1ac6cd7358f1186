# round 5 GPU call P: 512-thread forward blocks for the 1536-point 3 * 2^k rows (64-B segments),
# 512-thread row-inverse blocks for all ungrouped 3 * 2^k rows: the GPU suite, R / R^T op times,
# compute_kn phases and the C2 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r5p_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5p_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r5p_pytest_gpu.log
for cfg in "1024,1024 32 RT" "1024,1024 32 R" "2048,2048 200 RT" "4096,4096 25 RT"; do
  set -- $cfg
  timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op $3 2>/dev/null || exit 1
done | tee gpurun_out/r5p_passtime.txt
timeout -k 10 600 python tools/kn_phases.py --only C2,C3,C4,C5 2>/dev/null | tee gpurun_out/r5p_kn_phases.txt
timeout -k 10 600 python bench.py > gpurun_out/r5p_bench.json 2> gpurun_out/r5p_bench.err || { tail -20 gpurun_out/r5p_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r5p_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('pcg_wall_clock_ms'))"
