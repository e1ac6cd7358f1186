#!/bin/bash
# Block-shape variants of libhipgp for tuning: build here (BUILD=1), time on the GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
declare -A V
V[a]=""
V[b]="-DHGP_CONTIG_THREADS=256"
V[c]="-DHGP_CONTIG_THREADS=256 -DHGP_ROWT_PAIRS=4"
V[d]="-DHGP_ROWT_PAIRS=4"
if [ -n "$BUILD" ]; then
  for k in "${!V[@]}"; do make -s -C hipgp_amd/csrc VARIANT=$k VFLAGS="${V[$k]}" -j4 & done; wait
  exit 0
fi
mkdir -p gpurun_out
for k in $(echo "${!V[@]}" | tr ' ' '\n' | sort); do
  HGP_LIB=$PWD/hipgp_amd/libhipgp_$k.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --pcg-reps 2 ${BENCH_ARGS:-} > gpurun_out/var_$k.json 2> gpurun_out/var_$k.err || { echo "$k failed"; tail -5 gpurun_out/var_$k.err; exit 1; }
  python - "$k" "${V[$k]}" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/var_{sys.argv[1]}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], sys.argv[2], "| value", round(d["value"]), "frac", round(r["frac"], 3), "pcg_ms", round(d["pcg_wall_clock_ms"], 2),
      "passes", [(p["ms"], p["gbs"]) for p in r["passes"]])
PY
done
