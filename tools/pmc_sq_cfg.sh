#!/bin/bash
# SQ issue / stall counters of one operator's pass kernels at a config shape (passtime --op-only),
# one rocprofv3 --pmc pass per counter set, kernel-trace only:
#   SHAPE=256,256,128 RHS=25 TAG=C5 bash tools/pmc_sq_cfg.sh
# PCG=n: the kernels of n batched PCG(20) solves instead (the fused epilogues)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sq_$TAG
rm -rf $OUT; mkdir -p $OUT
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- \
    python3 tools/passtime.py --dims $SHAPE --rhs ${RHS:-25} --op ${OP:-K} ${PCG:+--pcg-only $PCG} --op-only 5 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT | tee $OUT/summary.txt
