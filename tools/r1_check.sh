#!/bin/bash
# GPU check: GPU tests, the bench line, optionally the SQ counters of the K-matvec passes
# (SQ=1) and the Infinity-Cache chunk sweep (WS_LIST="...").  Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
tail -1 gpurun_out/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', round(d['value']), 'frac', round(r['frac'],3), 'pcg_ms', round(d['pcg_wall_clock_ms'],2), d['pcg'], [(p['ms'], p['gbs']) for p in r['passes']], 'cpu', d.get('cpu_baseline', {}).get('value'))"
if [ -n "$SQ" ]; then bash tools/pmc_kop_sq.sh | grep -E "^[a-z]|VALU|WAVE_CYCLES|WAIT|BUSY|IDX" || exit $?; fi
if [ -n "$WS_LIST" ]; then bash tools/ws_sweep.sh; fi
exit 0
