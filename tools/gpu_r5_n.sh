# round 5 GPU call N: 512-thread row-inverse blocks for the ungrouped 3 * 2^k rows (C2 / C3 R / R^T,
# variant v512) against the default 1024; and the C4 R^T op at an 8 GiB workspace (fewer spectrum
# re-reads per op).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libhipgp libhipgp_v512; do
  for cfg in "2048,2048 200 RT" "2048,2048 200 R" "1024,1024 32 RT" "1024,1024 32 R"; do
    set -- $cfg
    HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op $3 2>/dev/null | sed "s/^/$lib /" || exit 1
  done
done | tee gpurun_out/r5n_tri_inv_threads.txt
for ws in 2048 8192; do
  HGP_WS_MB=$ws timeout -k 10 180 python tools/passtime.py --dims 4096,4096 --rhs 25 --op RT 2>/dev/null | sed "s/^/ws$ws /" || exit 1
done | tee -a gpurun_out/r5n_tri_inv_threads.txt
HGP_LIB=$PWD/hipgp_amd/libhipgp_v512.so timeout -k 10 600 python -u -m pytest tests/test_large_gpu.py tests/test_parity_gpu.py -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r5n_pytest_v512.log 2>&1; tail -3 gpurun_out/r5n_pytest_v512.log
