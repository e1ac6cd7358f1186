#!/bin/bash
# C5 config line at several workspace budgets / stream counts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/passtime.py --dims 256,256,128 --rhs 25 --op K || exit 1
for ws in default 4096; do
  if [ $ws = default ]; then unset HGP_WS_MB; else export HGP_WS_MB=$ws; fi
  timeout -k 10 300 python -u tools/bench_configs.py --only C5 > gpurun_out/c5_ws$ws.jsonl 2> gpurun_out/c5_ws$ws.err || { tail -20 gpurun_out/c5_ws$ws.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/c5_ws$ws.jsonl').read().splitlines()[-1]);print('$ws', d['kmatvec_batched_ms'], d['compute_kn_s'], d['compute_kn_hbm_frac'], d['peak_mem_gb'])"
done
