#!/bin/bash
# One GPU session: GPU tests, smoke, bench.  Every GPU step has its own time limit; a crash,
# abort or time-out (exit >= 124 / 134 / 139) ends the session immediately.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_if_fatal() {   # $1 = exit code, $2 = step
  local rc=$1
  echo "[session] $2 exit=$rc"
  if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then
    echo "[session] fatal exit from $2 -> stopping"; exit "$rc"; fi
}
STEPS="${1:-tests,smoke,bench}"
if [[ "$STEPS" == *tests* ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  stop_if_fatal $? pytest
  tail -25 gpurun_out/pytest_gpu.log
fi
if [[ "$STEPS" == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  stop_if_fatal $? smoke
  tail -3 gpurun_out/smoke.log
fi
if [[ "$STEPS" == *bench* ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  stop_if_fatal $? bench
  tail -3 gpurun_out/bench.log
fi
exit 0
