#!/bin/bash
# quick check: bench (per-pass times) + the parity / CG / large-grid GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { tail -20 gpurun_out/bench_q.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_q.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 4), "frac", round(r["frac"], 3),
      "ev_ms", round(r["event_op_ms"], 4), "pcg_ms", round(d["pcg_wall_clock_ms"], 2), "passes", [(p["ms"], p["gbs"]) for p in r["passes"]])
PY
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_q.log 2>&1 || { tail -40 gpurun_out/pytest_q.log; exit 1; }
tail -1 gpurun_out/pytest_q.log
