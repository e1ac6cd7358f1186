# round 3 GPU call C: the GPU test suite on the default build (tri lengths + folding + slab
# A2A receive + interleaved grouped conv blocks), then per-pass times at C4 / C3:
#   default     : G = 4 (4096-point rows) / 2 (2048), LAY_GRP* conv blocks
#   grpoff      : the same with the position-fast grouped conv (HGP_GRP_BLOCKS=0)
#   m3          : H >= 2048 contiguous conv lines at 3 waves / SIMD (no VGPR spills)
#   g2          : G = 2 for 4096-point rows + m3
# and the C5 R^T / R / K ops with 3*2^k lengths vs power-of-two lengths (HGP_LR=pow2)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_c.log 2>&1; rc=$?
tail -40 gpurun_out/pytest_gpu_c.log
[ $rc -le 1 ] || exit $rc
for v in default grpoff m3 g2; do
  lib=$PWD/hipgp_amd/libhipgp.so; env=""
  case $v in grpoff) env="HGP_GRP_BLOCKS=0";; m3|g2) lib=$PWD/hipgp_amd/libhipgp_$v.so;; esac
  for dr in 4096,4096:25 2048,2048:32 1024,1024:32; do
    d=${dr%%:*}; r=${dr#*:}
    echo -n "$v "
    env $env HGP_LIB=$lib timeout -k 10 120 python tools/passtime.py --dims $d --rhs $r || exit 1
  done
done 2>&1 | tee gpurun_out/r3_c_passtime.txt || exit 1
for lr in tri pow2; do
  for op in RT R K; do
    echo -n "C5 $op L_R=$lr "
    HGP_LR=$lr timeout -k 10 120 python tools/passtime.py --dims 256,256,128 --rhs 25 --op $op || exit 1
  done
done 2>&1 | tee -a gpurun_out/r3_c_passtime.txt || exit 1
timeout -k 10 300 python tools/c3_step.py 2>&1 | tee gpurun_out/r3_c3_step.jsonl || exit 1
exit $rc
