# round 5 GPU call T: one row pair per row-inverse block at the 4096-point rows (variant k1,
# HGP_ROWG_PAIRS_LONG_INV=1) against the default two: C4 K / C^-1 op times, C4 compute_kn phases,
# the full-size parity tests on the variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libhipgp libhipgp_k1 libhipgp libhipgp_k1; do
  for op in K CINV; do
    HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 180 python tools/passtime.py --dims 4096,4096 --rhs 25 --op $op 2>/dev/null | sed "s/^/$lib /" || exit 1
  done
  HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 300 python tools/kn_phases.py --only C4 2>/dev/null | sed "s/^/$lib /" || exit 1
done | tee gpurun_out/r5t_rowinv4096.txt

