#!/bin/bash
# rocprofv3 kernel stats + HBM traffic (FETCH_SIZE / WRITE_SIZE, one pass each) of one batched
# operator at a config shape:  SHAPE=4096,4096 RHS=25 TAG=C4 bash tools/prof_cfg.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
rm -rf $OUT; mkdir -p $OUT
NOPS=${NOPS:-10}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
  python3 tools/passtime.py --dims $SHAPE --rhs $RHS --op ${OP:-K} > $OUT/stats.log 2>&1 || { echo "stats failed"; tail -5 $OUT/stats.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- \
    python3 tools/passtime.py --dims $SHAPE --rhs $RHS --op ${OP:-K} --op-only $NOPS > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $OUT/$c.log; exit 1; }
done
LR=$(grep -o '"L_R": \[[0-9, ]*\]' $OUT/stats.log | head -1 | tr -d '"L_R: []')
python3 tools/pmc_cfg_summary.py $OUT $NOPS "$SHAPE" $RHS ${OP:-K} "$LR" | tee $OUT/summary.txt
