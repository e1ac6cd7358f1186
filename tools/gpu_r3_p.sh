# round 3 GPU call P: tg4 = grouped columns (G = 4: 2 pairs x 4 columns = 128-B segments) for the
# 6144-point (3 * 2^11) rows of the 2-D R / R^T at 4096-point axes.  GPU tests on tg4, C4 R^T / R
# passes and compute_kn phases against the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
HGP_LIB=$PWD/hipgp_amd/libhipgp_tg4.so timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_p.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu_p.log
[ $rc -le 1 ] || exit $rc
for lib in libhipgp libhipgp_tg4; do
  for op in RT R; do
    HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 120 python tools/passtime.py --dims 4096,4096 --rhs 25 --op $op | sed "s/^/$lib /" || exit 1
  done
  HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 600 python tools/kn_phases.py --only C4 | sed "s/^/$lib /" || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_p.txt || exit 1
exit $rc
