# round 4 GPU call AA: G = 4 grouped columns for the 2048-point rows (C3) vs the default G = 2,
# K and C^-1 ops at C3 (200 RHS), twice each; parity of the variant on the 2-D tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/hipgp_amd/libhipgp_g4.so
for r in 1 2; do
  for lib in base g4; do
    if [ $lib = g4 ]; then export HGP_LIB=$V; else unset HGP_LIB; fi
    for op in K CINV; do
      timeout -k 10 120 python tools/passtime.py --dims 2048,2048 --rhs 200 --op $op 2>/dev/null | sed "s/^/$lib /" || exit 1
    done
  done
done | tee gpurun_out/g4_aa.txt || exit 1
HGP_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_large_gpu.py tests/test_pcg_break_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_aa.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_aa.log; exit $rc
