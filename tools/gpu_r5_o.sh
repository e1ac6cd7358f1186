# round 5 GPU call O: 512-thread row-inverse blocks for the ungrouped 3 * 2^k rows as the default
# (the GPU suite), and the same for the forward pass (variant f512) at C2 / C3 R / R^T.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libhipgp libhipgp_f512; do
  for cfg in "2048,2048 200 RT" "2048,2048 200 R" "1024,1024 32 RT" "1024,1024 32 R"; do
    set -- $cfg
    HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op $3 2>/dev/null | sed "s/^/$lib /" || exit 1
  done
done | tee gpurun_out/r5o_tri_fwd_threads.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r5o_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5o_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r5o_pytest_gpu.log
