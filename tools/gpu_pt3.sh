#!/bin/bash
# per-pass times of the 3-D operators (C5 grid), 1 vs 2 streams
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for op in K RT; do
  timeout -k 10 120 python -u tools/passtime.py --dims ${DIMS:-256,256,128} --rhs 25 --op $op || exit 1
done
HGP_STREAMS=1 timeout -k 10 120 python -u tools/passtime.py --dims ${DIMS:-256,256,128} --rhs 25 --op K || exit 1
