# round 5 GPU call W: smaller row-inverse blocks at the C2 (1024-point, 4 pairs) and C3 (2048-point,
# 2 pairs) rows, variant h, against the default: the C2 headline op (bench --kop-only), C2 / C3 K
# pass times, compute_kn phases; alternated twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libhipgp libhipgp_h libhipgp libhipgp_h; do
  HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 180 python bench.py --kop-only --steps 50 --warmup 5 2>/dev/null | sed "s/^/$lib /" || exit 1
  for cfg in "1024,1024 32" "2048,2048 200"; do
    set -- $cfg
    HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op K 2>/dev/null | sed "s/^/$lib /" || exit 1
  done
  HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 300 python tools/kn_phases.py --only C2,C3 2>/dev/null | sed "s/^/$lib /" || exit 1
done | tee gpurun_out/r5w_rowinv_small.txt
HGP_LIB=$PWD/hipgp_amd/libhipgp_h.so timeout -k 10 600 python -u -m pytest tests/test_large_gpu.py tests/test_parity_gpu.py tests/test_cg_gpu.py -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r5w_pytest_h.log 2>&1; tail -3 gpurun_out/r5w_pytest_h.log
