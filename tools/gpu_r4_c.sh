# round 4 GPU call C: the whole GPU suite on the restored epilogue + new tests; R^T at C4 / C3 / C2
# with the power-of-two real-spectrum L_R (HGP_LR=pow2) against the 3*2^k complex default; bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_c.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" gpurun_out/pytest_gpu_c.log | tail -20; [ $rc -le 1 ] || exit 1
grep -E "C5 config-5|step [0-9] .me" gpurun_out/pytest_gpu_c.log | head -20
timeout -k 10 600 python -u -m pytest tests/test_fit_c3_gpu.py tests/test_fullsize_c5_gpu.py::test_solve_C5_config5_hyperparameters -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_c3c5_c.log 2>&1
rc=$?; grep -E "C5 config-5|step [0-9]|passed|failed" gpurun_out/pytest_c3c5_c.log | tail -30; [ $rc -le 1 ] || exit 1
for lr in default pow2; do
  for cfg in "4096,4096 25" "2048,2048 200" "1024,1024 32"; do
    set -- $cfg
    if [ $lr = default ]; then
      timeout -k 10 120 python tools/passtime.py --dims $1 --rhs $2 --op RT || exit 1
    else
      HGP_LR=pow2 timeout -k 10 120 python tools/passtime.py --dims $1 --rhs $2 --op RT || exit 1
    fi
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/rt_lr_c.txt || exit 1
HGP_LR=pow2 timeout -k 10 120 python tools/passtime.py --dims 256,256,128 --rhs 25 --op RT 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/rt_lr_c.txt || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err || { tail -20 gpurun_out/bench_c.err; exit 1; }
tail -1 gpurun_out/bench_c.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['pcg_wall_clock_ms'], d['roofline']['frac'], d.get('strong')['ms'], d.get('elbo_step')['ms'])"
