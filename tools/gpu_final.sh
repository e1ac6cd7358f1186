#!/bin/bash
# Round-end evidence: GPU tests, the default bench line (with CPU baseline), rocprofv3 kernel
# stats of the bench, PMC HBM traffic of the K matvec.  Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.json
bash tools/profile.sh ${TAG:-final} || exit 1
bash tools/pmc_kop.sh > gpurun_out/pmc_kop.log 2>&1 || { tail -20 gpurun_out/pmc_kop.log; exit 1; }
grep traffic_bytes_per_op gpurun_out/pmc_kop/pmc_kop_C2.json
