#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in 1024,1024:32 2048,2048:200 4096,4096:25 256,256,128:25; do
  timeout -k 10 200 python tools/passtime.py --dims ${s%%:*} --rhs ${s#*:} || exit 1
done
SHAPE=4096,4096 RHS=25 TAG=C4 bash tools/prof_cfg.sh || exit 1
SHAPE=256,256,128 RHS=25 TAG=C5 bash tools/prof_cfg.sh || exit 1
