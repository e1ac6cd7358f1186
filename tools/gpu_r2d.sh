#!/bin/bash
# strided-block variants at C5 (and C3 3-D slice), workspace budget at C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in libhipgp libhipgp_c16 libhipgp_c32 libhipgp_c64 libhipgp_c16w4; do
  echo -n "[$v] "; HGP_LIB=$PWD/hipgp_amd/$v.so timeout -k 10 120 python tools/passtime.py --dims 256,256,128 --rhs 25 || exit 1
done
for ws in 1024 2048 4096; do
  echo -n "[ws$ws] "; HGP_WS_MB=$ws timeout -k 10 120 python tools/passtime.py --dims 4096,4096 --rhs 25 || exit 1
done
