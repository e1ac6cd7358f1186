# round 5 GPU call E: (1) chained PCG (EPI_RF with the sequential forward tail) on / off:
# compute_kn phases at C2-C4, twice; (2) quad-layout variants of the C4 K / C^-1 / R^T ops and
# the C3 K op (main = 2 lines per 4096-point block at 4 waves/SIMD; q1m3 / q1m4 = 1 line at 3 / 4;
# noq = the plain G = 4 order of round 4).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for c in 1 0; do
    HGP_CHAIN_PCG=$c timeout -k 10 400 python tools/kn_phases.py --only C2,C3,C4 2>/dev/null | sed "s/^/chain$c /" || exit 1
  done
done | tee gpurun_out/r5e_kn_phases.txt
for v in main q1m3 q1m4 noq; do
  lib=$PWD/hipgp_amd/libhipgp.so; [ $v != main ] && lib=$PWD/hipgp_amd/libhipgp_$v.so
  for cfg in "4096,4096 25 K" "4096,4096 25 CINV" "4096,4096 25 RT" "2048,2048 200 K"; do
    set -- $cfg
    HGP_LIB=$lib timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op $3 2>/dev/null | sed "s/^/$v /" || exit 1
  done
done | tee gpurun_out/r5e_quad_variants.txt
