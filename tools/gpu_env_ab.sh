#!/bin/bash
# A/B of run-time knobs on one box: ENVS="name:VAR=val,VAR=val ..." (two reps, interleaved)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for v in $ENVS; do
  k=${v%%:*}; e=${v#*:}; e=${e//,/ }
  env $e timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 --warmup 10 --pcg-reps 3 ${BENCH_ARGS:-} > gpurun_out/env_$k.json 2> gpurun_out/env_$k.err || { echo "$k failed"; tail -5 gpurun_out/env_$k.err; exit 1; }
  python3 - "$k" <<'PY'
import json, sys
k = sys.argv[1]
d = json.loads(open(f"gpurun_out/env_{k}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{k:10s} value {round(d['value'])} ms/step {d['ms_per_step']:.4f} frac {r['frac']:.3f} pcg_ms {d['pcg_wall_clock_ms']:.2f} passes",
      [(p["ms"], p["gbs"]) for p in r["passes"]], flush=True)
PY
done
done
