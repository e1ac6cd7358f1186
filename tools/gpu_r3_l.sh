# round 3 GPU call L: li3 = line-inverse pass at 3 waves/SIMD; ld = buffer loads with drop offsets in
# the row / line forward passes of several lines per wave.  GPU tests on ld, per-pass times.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
HGP_LIB=$PWD/hipgp_amd/libhipgp_ld.so timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_l.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu_l.log
[ $rc -le 1 ] || exit $rc
for lib in libhipgp libhipgp_li3 libhipgp_ld; do
  for cfg in 256,256,128:25:K 256,256,128:25:RT 1024,1024:32:K 2048,2048:200:K; do
    d=${cfg%%:*}; rest=${cfg#*:}; r=${rest%%:*}; op=${rest#*:}
    HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 120 python tools/passtime.py --dims $d --rhs $r --op $op | sed "s/^/$lib /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_l_passtime.txt || exit 1
exit $rc
