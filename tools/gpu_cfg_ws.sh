#!/bin/bash
# C2-C5 K matvec and compute_kn against the byte model for several workspace budgets
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for ws in ${WS_LIST:-1024 136}; do
  HGP_WS_MB=$ws timeout -k 10 300 python tools/bench_configs.py --only ${ONLY:-C2,C3,C4,C5} > gpurun_out/cfg_ws$ws.jsonl 2> gpurun_out/cfg_ws$ws.err || { tail -5 gpurun_out/cfg_ws$ws.err; exit 1; }
  python3 - $ws <<'PY'
import json, sys
for l in open(f"gpurun_out/cfg_ws{sys.argv[1]}.jsonl"):
    d = json.loads(l)
    if "kmatvec_batched_ms" in d:
        print(sys.argv[1], d["config"], "B", d["B"], "Kop ms %.3f frac %.3f | compute_kn s %.4f model %.4f frac %.3f" % (
            d["kmatvec_batched_ms"], d["kmatvec_hbm_frac"], d["compute_kn_s"], d["compute_kn_model_s"], d["compute_kn_hbm_frac"]), flush=True)
PY
done
