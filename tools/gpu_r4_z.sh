# round 4 GPU call Z: the grouped-column conv as one block per (group, RHS) (HGP_GRP_BLOCKS=1,
# LAY_GRP*: whole 32-B units per block, no partial-line writes) vs G position-fast blocks, on the
# packed-fp32 build: K op at C4 / C3, twice each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for g in 0 1; do
    for cfg in "4096,4096 25" "2048,2048 200"; do
      set -- $cfg
      HGP_GRP_BLOCKS=$g timeout -k 10 120 python tools/passtime.py --dims $1 --rhs $2 --op K 2>/dev/null | sed "s/^/grp$g /" || exit 1
    done
  done
done | tee gpurun_out/grp_z.txt
