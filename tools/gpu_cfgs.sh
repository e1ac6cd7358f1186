#!/bin/bash
# C2 bench line (no CPU baseline) + the C5 / C4 config lines + compute_kn phases
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { tail -20 gpurun_out/bench_q.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_q.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("value", round(d["value"]), "ms/step", round(d["ms_per_step"], 4), "frac", round(r["frac"], 3),
      "pcg_ms", round(d["pcg_wall_clock_ms"], 2), "passes", [(p["ms"], p["gbs"]) for p in r["passes"]])
PY
timeout -k 10 400 python -u tools/bench_configs.py --only ${CFGS:-C5,C4} > gpurun_out/cfg_q.jsonl 2> gpurun_out/cfg_q.err || { tail -20 gpurun_out/cfg_q.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/cfg_q.jsonl"):
    d = json.loads(l)
    if "kmatvec_batched_ms" not in d: print(d["config"], d.get("gram_solve_s")); continue
    print(d["config"], "kmatvec_ms", round(d["kmatvec_batched_ms"], 3), "frac", round(d["kmatvec_hbm_frac"], 3),
          "compute_kn_s", round(d["compute_kn_s"], 4), "frac", round(d["compute_kn_hbm_frac"], 3), "peak_gb", round(d["peak_mem_gb"], 1))
PY
timeout -k 10 300 python -u tools/kn_phases.py --only ${CFGS:-C5,C4} || exit 1
