#!/bin/bash
# Round-2 session b: new GPU tests (a11 CG paths, C3/C4 PCG + ELBO, hyper-parameter grads),
# VALU-rate calibration.  Each GPU step has its own limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/valu_rate.bin > gpurun_out/valu_rate.txt 2>&1; cat gpurun_out/valu_rate.txt
timeout -k 10 600 python -u -m pytest tests/test_cg_gpu.py tests/test_hyper_gpu.py tests/test_large_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_new.log 2>&1 || { tail -40 gpurun_out/pytest_new.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_new.log | tail -40
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
