# round 5 GPU call Q: SQ counters of the C4 K op's passes (quad order, one-line conv blocks) --
# where the 4096-point column pass waits.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
SHAPE=4096,4096 RHS=25 OP=K TAG=C4K bash tools/pmc_sq_cfg.sh > /dev/null && grep -A19 "hgp::k_" gpurun_out/pmc_sq_C4K/summary.txt
