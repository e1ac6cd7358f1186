# round 5 GPU call I: the 2-D workspace budget (HGP_WS_MB: RHS per chunk, so spectrum re-reads
# per op) at 1, 2, 4 and 8 GiB: C3 K (200 RHS), C4 K / C^-1 / R^T (25 RHS) op times, and
# compute_kn phases at C2-C4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for ws in 1024 2048 4096 8192; do
  for cfg in "2048,2048 200 K" "4096,4096 25 K" "4096,4096 25 CINV" "4096,4096 25 RT"; do
    set -- $cfg
    HGP_WS_MB=$ws timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op $3 2>/dev/null | sed "s/^/ws$ws /" || exit 1
  done
  HGP_WS_MB=$ws timeout -k 10 600 python tools/kn_phases.py --only C2,C3,C4 2>/dev/null | sed "s/^/ws$ws /" || exit 1
done | tee gpurun_out/r5i_ws.txt
