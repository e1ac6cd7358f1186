# round 3 GPU call T: s8 = sequential half transforms in the 2048-point column pass only (no spills
# at 4 waves/SIMD) against the default: C3 (200 RHS) and C2 K per-pass times, GPU tests on s8.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in libhipgp libhipgp_s8; do
    for cfg in 2048,2048:200 1024,1024:32; do
      HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 120 python tools/passtime.py --dims ${cfg%%:*} --rhs ${cfg#*:} --op K | sed "s/^/$lib /" || exit 1
    done
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_t_passtime.txt || exit 1
HGP_LIB=$PWD/hipgp_amd/libhipgp_s8.so timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_t.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_t.log
exit $rc
