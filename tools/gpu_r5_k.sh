# round 5 GPU call K: why the C4 R^T row inverse (12288-point rows) takes 2.3x its forward pass
# for the same bytes: SQ counters and per-kernel bytes of the R^T op at C4 (P = 24 build).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
SHAPE=4096,4096 RHS=25 OP=RT TAG=C4RT bash tools/pmc_sq_cfg.sh && \
SHAPE=4096,4096 RHS=25 OP=RT TAG=C4RT NOPS=3 bash tools/prof_cfg.sh
