#!/bin/bash
# Compile-time variants of libhipgp for tuning: build here (BUILD=1), time on the GPU box.
#   VARS="a: s8:-DHGP_ROWT_PAIRS=4"  (name:flags, space separated; flags use "," for spaces)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARS=${VARS:-"a:"}
if [ -n "$BUILD" ]; then
  for v in $VARS; do
    k=${v%%:*}; f=${v#*:}; f=${f//,/ }
    make -s -C hipgp_amd/csrc VARIANT=$k VFLAGS="$f" -j8 > /tmp/variant_$k.log 2>&1 &
  done
  wait
  ls -la hipgp_amd/libhipgp_*.so
  exit 0
fi
mkdir -p gpurun_out
for v in $VARS; do
  k=${v%%:*}
  HGP_LIB=$PWD/hipgp_amd/libhipgp_$k.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --pcg-reps 3 ${BENCH_ARGS:-} > gpurun_out/var_$k.json 2> gpurun_out/var_$k.err || { echo "$k failed"; tail -5 gpurun_out/var_$k.err; exit 1; }
  python3 - "$v" <<'PY'
import json, sys
k = sys.argv[1].split(":")[0]
d = json.loads(open(f"gpurun_out/var_{k}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], "| value", round(d["value"]), "frac", round(r["frac"], 3), "pcg_ms", round(d["pcg_wall_clock_ms"], 2),
      "passes", [(p["ms"], p["gbs"]) for p in r["passes"]], flush=True)
PY
done
