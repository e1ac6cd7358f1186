# round 5 GPU call Z: the C4 R^T op and compute_kn's R^T phase at 2 / 4 / 8 GiB workspaces (fewer
# re-reads of the complex R spectrum per op), alternated.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for ws in 2048 8192 4096 2048 8192; do
  HGP_WS_MB=$ws timeout -k 10 180 python tools/passtime.py --dims 4096,4096 --rhs 25 --op RT 2>/dev/null | sed "s/^/ws$ws /" || exit 1
  HGP_WS_MB=$ws timeout -k 10 300 python tools/kn_phases.py --only C4 2>/dev/null | sed "s/^/ws$ws /" || exit 1
done | tee gpurun_out/r5z_rt_ws.txt
