#!/bin/bash
# Sweep the per-op RHS-chunk workspace budget (HGP_WS_MB): small chunks keep the pass
# intermediates resident in the 256 MiB Infinity Cache between passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mb in ${WS_LIST:-1024 200 136 100 68}; do
  HGP_WS_MB=$mb timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --pcg-reps 2 ${BENCH_ARGS:-} > gpurun_out/ws_$mb.json 2> gpurun_out/ws_$mb.err || exit $?
  python - "$mb" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ws_{sys.argv[1]}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], "MB: value", round(d["value"]), "frac", round(r["frac"], 3), "pcg_ms", round(d["pcg_wall_clock_ms"], 2),
      "passes", [(p["ms"], p["gbs"]) for p in r["passes"]])
PY
done
