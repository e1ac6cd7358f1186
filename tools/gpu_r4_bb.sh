# round 4 GPU call BB: SQ issue / LDS counters of the C4 R^T passes on the final (packed-fp32) build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
SHAPE=4096,4096 RHS=25 TAG=C4RT_pk OP=RT timeout -k 10 600 bash tools/pmc_sq_cfg.sh > gpurun_out/pmc_sq_C4RT_pk.log 2>&1 || { tail -5 gpurun_out/pmc_sq_C4RT_pk.log; exit 1; }
grep -A20 "6144, 3, 4" gpurun_out/pmc_sq_C4RT_pk/summary.txt | head -22
