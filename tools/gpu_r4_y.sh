# round 4 GPU call Y: per-kernel HBM bytes (rocprofv3 FETCH_SIZE / WRITE_SIZE) and kernel stats of the
# K op at C4 and C3 and of R^T at C4 on the final (packed-fp32) build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
SHAPE=4096,4096 RHS=25 TAG=C4K_final OP=K timeout -k 10 600 bash tools/prof_cfg.sh > gpurun_out/prof_C4K_final.log 2>&1 || { tail -5 gpurun_out/prof_C4K_final.log; exit 1; }
tail -12 gpurun_out/prof_C4K_final.log
SHAPE=2048,2048 RHS=200 TAG=C3K_final OP=K timeout -k 10 600 bash tools/prof_cfg.sh > gpurun_out/prof_C3K_final.log 2>&1 || { tail -5 gpurun_out/prof_C3K_final.log; exit 1; }
tail -12 gpurun_out/prof_C3K_final.log
SHAPE=4096,4096 RHS=25 TAG=C4RT_final OP=RT timeout -k 10 600 bash tools/prof_cfg.sh > gpurun_out/prof_C4RT_final.log 2>&1 || { tail -5 gpurun_out/prof_C4RT_final.log; exit 1; }
tail -14 gpurun_out/prof_C4RT_final.log
