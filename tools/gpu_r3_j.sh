# round 3 GPU call J: the buffer-store row-inverse epilogue (libhipgp_ep: no VGPR spills at 4096) and
# P = 32 row passes (libhipgp_rp) against the default: GPU tests on ep, per-pass times, PMC of ep at C4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
HGP_LIB=$PWD/hipgp_amd/libhipgp_ep.so timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_j.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu_j.log
[ $rc -le 1 ] || exit $rc
for lib in libhipgp libhipgp_ep libhipgp_rp; do
  for cfg in 4096,4096:25:K 4096,4096:25:CINV 2048,2048:200:K 1024,1024:32:K 256,256,128:25:K; do
    d=${cfg%%:*}; rest=${cfg#*:}; r=${rest%%:*}; op=${rest#*:}
    HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 120 python tools/passtime.py --dims $d --rhs $r --op $op | sed "s/^/$lib /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_j_passtime.txt || exit 1
HGP_LIB=$PWD/hipgp_amd/libhipgp_ep.so SHAPE=4096,4096 RHS=25 TAG=C4_ep timeout -k 10 600 bash tools/prof_cfg.sh || exit 1
exit $rc
