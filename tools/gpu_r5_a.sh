# round 5 GPU call A: baseline on the round-4 final tree — bench line, per-pass times of the
# C2 / C4 K op and the C4 R^T op.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/r5a_bench.json 2> gpurun_out/r5a_bench.err || { tail -20 gpurun_out/r5a_bench.err; exit 1; }
tail -1 gpurun_out/r5a_bench.json
for cfg in "1024,1024 32 K" "4096,4096 25 K" "4096,4096 25 RT" "2048,2048 200 K"; do
  set -- $cfg
  timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op $3 2>/dev/null || exit 1
done | tee gpurun_out/r5a_passtime.txt
