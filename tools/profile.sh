#!/bin/bash
# rocprofv3 kernel-trace summary of the bench (timing pass) — run on the GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${1:-run}
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 --pcg-reps 1 > "$OUT/bench.log" 2>&1
rc=$?
echo "[profile] rocprofv3 exit=$rc"
find "$OUT" -name "*kernel_stats.csv" | head -3
f=$(find "$OUT" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -30 "$f"
exit $rc
