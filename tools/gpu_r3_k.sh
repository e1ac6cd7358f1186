# round 3 GPU call K: 3-D (C5) pass variants.  ep2 = branch-free buffer-store epilogues in the
# line / row inverse passes of several lines per wave; ms2 = ep2 + 3 waves/SIMD and 256-thread
# blocks for the H <= 512 column passes (no spills).  GPU tests on ms2, per-pass times, PMC at C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
HGP_LIB=$PWD/hipgp_amd/libhipgp_ms2.so timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_k.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu_k.log
[ $rc -le 1 ] || exit $rc
for lib in libhipgp libhipgp_ep2 libhipgp_ms2; do
  for cfg in 256,256,128:25:K 256,256,128:25:RT 1024,1024:32:K 4096,4096:25:K; do
    d=${cfg%%:*}; rest=${cfg#*:}; r=${rest%%:*}; op=${rest#*:}
    HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 120 python tools/passtime.py --dims $d --rhs $r --op $op | sed "s/^/$lib /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_k_passtime.txt || exit 1
for lib in libhipgp libhipgp_ms2; do
  HGP_LIB=$PWD/hipgp_amd/$lib.so SHAPE=256,256,128 RHS=25 TAG=C5_$lib timeout -k 10 600 bash tools/prof_cfg.sh || exit 1
done
exit $rc
