#!/bin/bash
# GPU check: tests, interleaved env A/B (ENVS), rocprof kernel stats of the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
ENVS="${ENVS:-HGP_STREAMS=1 HGP_STREAMS=2 HGP_STREAMS=1 HGP_STREAMS=2}" bash tools/env_sweep.sh || exit 1
[ -n "$NOPROF" ] || bash tools/profile.sh ${TAG:-r1b} || exit 1
