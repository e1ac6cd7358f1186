#!/bin/bash
# Per-pass timings of the 2-D K matvec at the larger configs (C3 2048^2, C4 4096^2) + kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in ${SPECS:-"2048:64" "4096:25"}; do
  m=${spec%%:*}; b=${spec#*:}
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 --pcg-reps 1 --m $m --rhs $b > gpurun_out/size_$m.json 2> gpurun_out/size_$m.err || { echo "m=$m failed"; tail -5 gpurun_out/size_$m.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/size_$m.json').read().strip().splitlines()[-1]); r=d['roofline']
print('m=$m B=$b', 'value', round(d['value']), 'frac', round(r['frac'],3), 'op_ms', round(r['op_ms'],3), 'pcg_ms', round(d['pcg_wall_clock_ms'],1), [(p['ms'], p['gbs']) for p in r['passes']], flush=True)"
  if [ -n "$PROF" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_size_$m -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kop-only --steps 10 --warmup 3 --m $m --rhs $b > gpurun_out/prof_size_$m.log 2>&1 || exit 1
    head -8 $(find gpurun_out/prof_size_$m -name "*kernel_stats.csv" | head -1) | cut -c1-150
  fi
done
