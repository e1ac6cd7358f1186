#!/bin/bash
# Bench the default library under several environment settings (one bench run each).
#   ENVS="HGP_STREAMS=1 HGP_STREAMS=2 HGP_STREAMS=3"   (',' joins several variables)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for e in ${ENVS:-HGP_STREAMS=1 HGP_STREAMS=2}; do
  i=$((i+1))
  env ${e//,/ } timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --pcg-reps 3 ${BENCH_ARGS:-} > gpurun_out/env_$i.json 2> gpurun_out/env_$i.err || { echo "$e failed"; tail -5 gpurun_out/env_$i.err; exit 1; }
  python3 - "$e" "$i" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/env_{sys.argv[2]}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], "| value", round(d["value"]), "frac", round(r["frac"], 3), "op_ms", round(r["op_ms"], 4), "pcg_ms", round(d["pcg_wall_clock_ms"], 2),
      "passes", [(p["ms"], p["gbs"]) for p in r["passes"]], flush=True)
PY
done
