#!/bin/bash
# A/B of library builds on one box: LIBS="name:path ..." (default: the in-tree build + variants)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -x tools/valu_rate.bin ] && [ -n "$VALU" ] && { timeout -k 10 60 ./tools/valu_rate.bin > gpurun_out/valu_rate.txt 2>&1; cat gpurun_out/valu_rate.txt; }
for rep in 1 2; do
for v in ${LIBS:-"main:hipgp_amd/libhipgp.so"}; do
  k=${v%%:*}; lib=${v#*:}
  HGP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 --warmup 10 --pcg-reps 3 ${BENCH_ARGS:-} > gpurun_out/ab_$k.json 2> gpurun_out/ab_$k.err || { echo "$k failed"; tail -5 gpurun_out/ab_$k.err; exit 1; }
  python3 - "$k" <<'PY'
import json, sys
k = sys.argv[1]
d = json.loads(open(f"gpurun_out/ab_{k}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{k:8s} value {round(d['value'])} ms/step {d['ms_per_step']:.4f} frac {r['frac']:.3f} pcg_ms {d['pcg_wall_clock_ms']:.2f} passes",
      [(p["ms"], p["gbs"]) for p in r["passes"]], flush=True)
PY
done
done
