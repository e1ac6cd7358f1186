# round 5 evidence on the final tree (part B): the five-config table, compute_kn phases, per-pass
# times of R^T at C2-C5, per-kernel HBM bytes of the C4 K and R^T ops.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python tools/bench_configs.py > gpurun_out/configs_final.jsonl 2> gpurun_out/configs_final.err || { tail -5 gpurun_out/configs_final.err; exit 1; }
cut -c1-250 gpurun_out/configs_final.jsonl
timeout -k 10 600 python tools/kn_phases.py --only C2,C3,C4,C5 2>/dev/null | tee gpurun_out/kn_phases_final.jsonl || exit 1
for cfg in "1024,1024 32 RT" "2048,2048 200 RT" "4096,4096 25 RT" "256,256,128 25 RT" "4096,4096 25 K" "1024,1024 32 K"; do
  set -- $cfg
  timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op $3 2>/dev/null || exit 1
done | tee gpurun_out/passtime_final.txt
SHAPE=4096,4096 RHS=25 OP=K TAG=C4K_final NOPS=3 bash tools/prof_cfg.sh > /dev/null || exit 1
SHAPE=4096,4096 RHS=25 OP=RT TAG=C4RT_final NOPS=3 bash tools/prof_cfg.sh > /dev/null || exit 1
grep -h "per op\|traffic_over" gpurun_out/prof_C4K_final/summary.txt gpurun_out/prof_C4RT_final/summary.txt | cut -c1-200
