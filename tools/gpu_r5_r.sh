# round 5 GPU call R: radix-8 (P = 24) against radix-4 (P = 12, variant p12) stages in the 3 * 2^k
# contiguous fp32 passes, per line length: R^T at C2 (1536-point), C3 (3072), C4 (6144).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libhipgp libhipgp_p12; do
  for cfg in "1024,1024 32 RT" "2048,2048 200 RT" "4096,4096 25 RT"; do
    set -- $cfg
    HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op $3 2>/dev/null | sed "s/^/$lib /" || exit 1
  done
done | tee gpurun_out/r5r_tri_p.txt
