#!/bin/bash
# per-pass times of library variants at several grids (GPU box): VARS="a b" DIMS="4096,4096:25 1024,1024:32"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in ${VARS:-a}; do
  for dr in ${DIMS:-"4096,4096:25 1024,1024:32"}; do
    d=${dr%%:*}; r=${dr#*:}
    echo -n "$v "
    HGP_LIB=$PWD/hipgp_amd/libhipgp_$v.so timeout -k 10 120 python tools/passtime.py --dims $d --rhs $r ${OPARGS:-} || exit 1
  done
done
