# round 3 GPU call B: grouped-column 2-D intermediate (default build) vs the plain layout (g1),
# per-pass times at C2 / C3 / C4, then the GPU test suite on the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in g1 default; do
  lib=$PWD/hipgp_amd/libhipgp.so; [ $v = default ] || lib=$PWD/hipgp_amd/libhipgp_$v.so
  for dr in 4096,4096:25 2048,2048:32 1024,1024:32; do
    d=${dr%%:*}; r=${dr#*:}
    echo -n "$v "
    HGP_LIB=$lib timeout -k 10 120 python tools/passtime.py --dims $d --rhs $r || exit 1
  done
done 2>&1 | tee gpurun_out/r3_grouped_passtime.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_b.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu_b.log
exit $rc
