# round 5 GPU call AA: radix-8 stages (24 points a thread) in the grouped 12288-point row passes of
# the C4 R / R^T (variant r24) against radix-4 (12): op / pass times alternated, C4 compute_kn
# phases, and the parity tests that reach those rows on the variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libhipgp libhipgp_r24 libhipgp libhipgp_r24; do
  for op in RT R; do
    HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 180 python tools/passtime.py --dims 4096,4096 --rhs 25 --op $op 2>/dev/null | sed "s/^/$lib /" || exit 1
  done
  HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 300 python tools/kn_phases.py --only C4 2>/dev/null | sed "s/^/$lib /" || exit 1
done | tee gpurun_out/r5aa_rows_p24.txt
HGP_LIB=$PWD/hipgp_amd/libhipgp_r24.so timeout -k 10 600 python -u -m pytest tests/test_large_gpu.py tests/test_parity_gpu.py tests/test_grad_gpu.py -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r5aa_pytest_r24.log 2>&1; tail -3 gpurun_out/r5aa_pytest_r24.log
