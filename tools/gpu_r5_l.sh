# round 5 GPU call L: one row pair per block for the 12288-point (3 * 2^k) rows of the C4 R / R^T
# (HGP_ROWG_PAIRS_TRI=1, variant t1) against the default two: op / pass times, the C4 B = 200
# parity test and the R^T parity cases on the variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libhipgp libhipgp_t1; do
  for op in RT R; do
    HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 180 python tools/passtime.py --dims 4096,4096 --rhs 25 --op $op 2>/dev/null | sed "s/^/$lib /" || exit 1
  done
done | tee gpurun_out/r5l_tri_pairs.txt
HGP_LIB=$PWD/hipgp_amd/libhipgp_t1.so timeout -k 10 600 python -u -m pytest tests/test_large_gpu.py tests/test_long_axis_gpu.py -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r5l_pytest_t1.log 2>&1; tail -3 gpurun_out/r5l_pytest_t1.log
