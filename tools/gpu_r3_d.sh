# round 3 GPU call D: the GPU test suite (slab A2A stage, fp64 long axes incl. the full-grid
# R / R^T route, C5 full size), per-pass times of the 4096 / 2048-point row variants:
#   default : G = 4 (4096-point rows, LAY_CONTIG_G conv) / 2 (2048)
#   p1      : plain layout for 4096-point rows
#   p1m3    : p1 + H >= 2048 contiguous conv lines at 3 waves / SIMD (no VGPR spills)
#   m3      : default + the same
# the C5 R^T / K ops at 3-D workspace budgets of 1 / 4 (default) / 8 GiB, and the C3 minibatch step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_d.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu_d.log
[ $rc -le 1 ] || exit $rc
for v in default p1 p1m3 m3; do
  lib=$PWD/hipgp_amd/libhipgp.so; [ $v = default ] || lib=$PWD/hipgp_amd/libhipgp_$v.so
  for dr in 4096,4096:25 2048,2048:32 1024,1024:32; do
    d=${dr%%:*}; r=${dr#*:}
    echo -n "$v "
    HGP_LIB=$lib timeout -k 10 120 python tools/passtime.py --dims $d --rhs $r || exit 1
  done
done 2>&1 | tee gpurun_out/r3_d_passtime.txt || exit 1
for ws in 1024 default 8192; do
  for op in RT K; do
    echo -n "C5 $op ws=$ws "
    if [ $ws = default ]; then
      timeout -k 10 120 python tools/passtime.py --dims 256,256,128 --rhs 25 --op $op || exit 1
    else
      HGP_WS_MB=$ws timeout -k 10 120 python tools/passtime.py --dims 256,256,128 --rhs 25 --op $op || exit 1
    fi
  done
done 2>&1 | tee -a gpurun_out/r3_d_passtime.txt || exit 1
timeout -k 10 300 python tools/c3_step.py 2>&1 | tee gpurun_out/r3_c3_step.jsonl || exit 1
exit $rc
