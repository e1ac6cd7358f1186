#!/bin/bash
# run-to-run spread of the C2 bench line on one box: ms_per_step (timed loop) vs event_op_ms
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for i in 1 2 3; do
  for g in 1 0; do
    HGP_GRAPH=$g timeout -k 10 120 python bench.py --no-cpu-baseline --pcg-reps 1 ${BARGS:-} > gpurun_out/bv.json 2> gpurun_out/bv.err || { tail -5 gpurun_out/bv.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/bv.json').read().strip().splitlines()[-1]); r=d['roofline']
print('graph=$g', round(d['value']), 'ms/step', round(d['ms_per_step'],4), 'ev', round(r['event_op_ms'],4))"
  done
done
