# round 5 GPU call Y: 1024-point column lines of two waves (8 points a thread, ~71 VGPRs, 6 waves
# per SIMD; variant c8) against one wave of 16 points: the C2 headline op (bench --kop-only), C2 K
# pass times, C2 compute_kn phases; alternated twice; parity tests on the variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libhipgp libhipgp_c8 libhipgp libhipgp_c8; do
  HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 180 python bench.py --kop-only --steps 50 --warmup 5 2>/dev/null | sed "s/^/$lib /" || exit 1
  HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 180 python tools/passtime.py --dims 1024,1024 --rhs 32 --op K 2>/dev/null | sed "s/^/$lib /" || exit 1
  HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 300 python tools/kn_phases.py --only C2 2>/dev/null | sed "s/^/$lib /" || exit 1
done | tee gpurun_out/r5y_conv1024_p8.txt
HGP_LIB=$PWD/hipgp_amd/libhipgp_c8.so timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_cg_gpu.py -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r5y_pytest_c8.log 2>&1; tail -3 gpurun_out/r5y_pytest_c8.log
