#!/bin/bash
# C2 bench with RHS chunks forced by the workspace budget (HGP_WS_MB; 8.4 MB per RHS, 2 streams)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for w in ${WS:-default 68 135 270 default}; do
  if [ "$w" = default ]; then unset HGP_WS_MB; else export HGP_WS_MB=$w; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --pcg-reps 1 > gpurun_out/ws_$w.json 2> gpurun_out/ws_$w.err || { tail -5 gpurun_out/ws_$w.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/ws_$w.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$w', round(d['value']), round(d['ms_per_step'],4), round(r['frac'],3), round(d['pcg_wall_clock_ms'],2))"
done
