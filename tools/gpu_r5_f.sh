# round 5 GPU call F: default build (quad order, one 4096-point line per block at 4 waves/SIMD;
# chained PCG off): GPU suite incl. the G19 nine-run bound, then one vs two RHS streams per op
# (HGP_STREAMS) at C2-C5: op times and compute_kn phases.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r5f_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5f_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r5f_pytest_gpu.log
grep -h "nine-run" -r gpurun_out/r5f_pytest_gpu.log | head -4
for ns in 2 1; do
  for cfg in "1024,1024 32 K" "2048,2048 200 K" "4096,4096 25 K" "4096,4096 25 RT" "256,256,128 25 K" "256,256,128 25 RT"; do
    set -- $cfg
    HGP_STREAMS=$ns timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op $3 2>/dev/null | sed "s/^/streams$ns /" || exit 1
  done
  HGP_STREAMS=$ns timeout -k 10 600 python tools/kn_phases.py --only C2,C3,C4,C5 2>/dev/null | sed "s/^/streams$ns /" || exit 1
done | tee gpurun_out/r5f_streams.txt
