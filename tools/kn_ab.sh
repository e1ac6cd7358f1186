#!/bin/bash
# A/B of library variants on compute_kn (PCG wall clock) at C2 (bench) and C5/C4 (kn_phases)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in ${VARS:-old new}; do
  HGP_LIB=$PWD/hipgp_amd/libhipgp_$v.so timeout -k 10 200 python tools/kn_phases.py --only ${CFGS:-C5,C4} > gpurun_out/kn_$v.log 2>&1 || { tail -5 gpurun_out/kn_$v.log; exit 1; }
  echo "$v $(grep -h '{' gpurun_out/kn_$v.log | tr '\n' ' ')"
done
