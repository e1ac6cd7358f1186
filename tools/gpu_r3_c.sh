# round 3 GPU call C: the GPU test suite on the default build (tri lengths + folding + slab
# A2A receive), then per-pass times: grouped G for 4096-point rows (default G=4 vs g2 build),
# and the C5 R^T op with 3*2^k lengths vs power-of-two lengths (HGP_LR=pow2)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_c.log 2>&1; rc=$?
tail -40 gpurun_out/pytest_gpu_c.log
for v in g2 default; do
  lib=$PWD/hipgp_amd/libhipgp.so; [ $v = default ] || lib=$PWD/hipgp_amd/libhipgp_$v.so
  for dr in 4096,4096:25 2048,2048:32; do
    d=${dr%%:*}; r=${dr#*:}
    echo -n "$v "
    HGP_LIB=$lib timeout -k 10 120 python tools/passtime.py --dims $d --rhs $r || exit 1
  done
done 2>&1 | tee gpurun_out/r3_c_passtime.txt
for lr in tri pow2; do
  for op in RT R K; do
    echo -n "C5 $op L_R=$lr "
    HGP_LR=$lr timeout -k 10 120 python tools/passtime.py --dims 256,256,128 --rhs 25 --op $op || exit 1
  done
done 2>&1 | tee -a gpurun_out/r3_c_passtime.txt
exit $rc
