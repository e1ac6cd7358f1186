# round 3 GPU call M: eq = the PCG row-inverse epilogues staged without per-position branches for
# rows of exactly H outputs (no spills at 4096).  compute_kn phases default vs eq; C5 R^T against the
# workspace budget (RHS per chunk: the complex spectrum is fetched once per chunk).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libhipgp libhipgp_eq; do
  HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 600 python tools/kn_phases.py --only C4,C5,C3,C2 | sed "s/^/$lib /" || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_m_kn_phases.txt || exit 1
for rep in 1 2; do
  for ws in 4096 8192 16384 26000; do
    HGP_LIB=$PWD/hipgp_amd/libhipgp_eq.so HGP_WS_MB=$ws timeout -k 10 120 python tools/passtime.py --dims 256,256,128 --rhs 25 --op RT | sed "s/^/ws=$ws /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_m_rt_ws.txt || exit 1
