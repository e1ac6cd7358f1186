#!/bin/bash
# HBM traffic of the batched K matvec (C2) from rocprofv3 PMC counters, one counter per pass
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950), kernel-trace only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_kop
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- \
    python3 bench.py --kop-only --settle-s 0 --steps 10 --warmup 3 > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; tail -20 $OUT/$c.log; exit 1; }
done
python3 tools/pmc_kop_summary.py $OUT $OUT/pmc_kop_C2.json 13
