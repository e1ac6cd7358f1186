#!/bin/bash
# rocprofv3 kernel-trace summary of the bench (timing pass) — run on the GPU box.
# Output under gpurun_out/prof_<tag>/ (copy the stats csv into profiles/ afterwards).
# BENCH_ARGS overrides the bench arguments, e.g. BENCH_ARGS="--kop-only --steps 50 --warmup 5"
# for a summary of the headline K matvec's kernels alone (no compute_kn / legs / other configs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- \
  python3 bench.py ${BENCH_ARGS:---no-cpu-baseline --steps 20 --warmup 5 --pcg-reps 2} > "$OUT/bench.log" 2>&1
rc=$?
echo "[profile] rocprofv3 exit=$rc"
f=$(find "$OUT" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -12 "$f" | cut -c1-200

exit $rc
