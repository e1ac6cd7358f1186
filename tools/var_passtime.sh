#!/bin/bash
# Variant libraries side by side on per-pass timings: VARS="a s8 ..." ("a" = default build),
# SHAPES="256,256,128:25 ..." ; BENCH=1 also runs the C2 bench line per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARS:-a}; do
  if [ "$v" = a ]; then L=$PWD/hipgp_amd/libhipgp.so; else L=$PWD/hipgp_amd/libhipgp_$v.so; fi
  for s in ${SHAPES:-256,256,128:25}; do
    echo -n "[$v] "; HGP_LIB=$L timeout -k 10 200 python tools/passtime.py --dims ${s%%:*} --rhs ${s#*:} || exit 1
  done
  if [ -n "$BENCH" ]; then
    HGP_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --pcg-reps 3 > gpurun_out/vb_$v.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/vb_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('[$v] C2 value', round(d['value']), 'frac', round(r['frac'],3), 'pcg_ms', round(d['pcg_wall_clock_ms'],2), 'setup_ms', round(d['pcg']['setup_ms'],2), [p['ms'] for p in r['passes']], flush=True)"
  fi
done
