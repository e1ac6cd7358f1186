# round 4 GPU call T: 2-D workspace budget (RHS per chunk) re-swept on the packed-fp32 build, K op
# at C4 (25 RHS) and C3 (200 RHS).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for ws in 512 768 1024 1536 2048; do
  for cfg in "4096,4096 25" "2048,2048 200"; do
    set -- $cfg
    HGP_WS_MB=$ws timeout -k 10 120 python tools/passtime.py --dims $1 --rhs $2 --op K 2>/dev/null | sed "s/^/ws$ws /" || exit 1
  done
done | tee gpurun_out/ws_t.txt
