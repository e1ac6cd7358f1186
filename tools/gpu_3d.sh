#!/bin/bash
# 3-D path check: per-pass times (C5 grid), the GPU test suite, then the C5 / C4 config lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for op in K RT; do
  timeout -k 10 120 python -u tools/passtime.py --dims ${DIMS:-256,256,128} --rhs 25 --op $op || exit 1
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_3d.log 2>&1 || { tail -40 gpurun_out/pytest_3d.log; exit 1; }
tail -1 gpurun_out/pytest_3d.log
timeout -k 10 400 python -u tools/bench_configs.py --only ${CFGS:-C5,C4} > gpurun_out/cfg_3d.jsonl 2> gpurun_out/cfg_3d.err || { tail -20 gpurun_out/cfg_3d.err; exit 1; }
cat gpurun_out/cfg_3d.jsonl
timeout -k 10 300 python -u tools/kn_phases.py --only C5,C4 || exit 1
