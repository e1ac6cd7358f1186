#!/bin/bash
# SQ issue counters of the K-matvec passes for several library builds on one box
# (LIBS="name:path ..."), one rocprofv3 --pmc pass per build, kernel-trace only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SET=${SET:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"}
for v in $LIBS; do
  k=${v%%:*}; lib=${v#*:}
  OUT=gpurun_out/pmc_ab_$k
  rm -rf $OUT; mkdir -p $OUT
  HGP_LIB=$PWD/$lib timeout -s KILL 90 rocprofv3 --pmc $SET --output-format csv -d $OUT/p -o run -- \
    python3 bench.py --kop-only --steps 5 --warmup 2 ${BENCH_ARGS:-} > $OUT/log.txt 2>&1 || { echo "pmc $k failed"; tail -5 $OUT/log.txt; exit 1; }
  echo "== $k"; python3 tools/pmc_summary.py $OUT | grep -A12 "hgp::" | tee $OUT/summary.txt
done
