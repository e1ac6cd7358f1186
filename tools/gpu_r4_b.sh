# round 4 GPU call B: the slab PCG on device buffers (2 / 3 same-device ranks), the G19 config-3
# fit tests, plan memory accounting; R^T chunk-size sweep at C4 / C3 / C2 (spectrum re-reads);
# SQ counters of the fused PCG epilogues at C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_slab_gpu.py tests/test_fit_c3_gpu.py tests/test_long_axis_gpu.py tests/test_model_gpu.py "tests/test_fullsize_c5_gpu.py::test_solve_C5_config5_hyperparameters" -v --timeout 300 --timeout-method thread > gpurun_out/pytest_b.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error" gpurun_out/pytest_b.log | tail -40; [ $rc -le 1 ] || exit 1
for ws in 0 2048 4096 8192 16384; do
  for cfg in "4096,4096 25" "2048,2048 200" "1024,1024 32"; do
    set -- $cfg
    if [ $ws = 0 ]; then
      timeout -k 10 120 python tools/passtime.py --dims $1 --rhs $2 --op RT || exit 1
    else
      HGP_WS_MB=$ws timeout -k 10 120 python tools/passtime.py --dims $1 --rhs $2 --op RT || exit 1
    fi
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/rt_ws_b.txt || exit 1
SHAPE=1024,1024 RHS=32 TAG=C2pcg PCG=3 timeout -k 10 600 bash tools/pmc_sq_cfg.sh > gpurun_out/pmc_sq_C2pcg.log 2>&1 || { tail -5 gpurun_out/pmc_sq_C2pcg.log; exit 1; }
grep -A18 "row_inv" gpurun_out/pmc_sq_C2pcg/summary.txt | head -80
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || { tail -20 gpurun_out/bench_b.err; exit 1; }
tail -1 gpurun_out/bench_b.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['pcg_wall_clock_ms'], d.get('strong'), d.get('elbo_step'))"
