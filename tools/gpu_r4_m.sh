# round 4 GPU call M: is the C2 column pass quantised in rounds of resident blocks?  Per-pass times of
# the K op at 1024^2 for 1..8, 12, 16, 32 RHS (chunks of <= 8 RHS; a pass-isolated chunk of Q RHS is
# 1025 Q lines in blocks of 8, two blocks per CU).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3 4 5 6 7 8 12 16 32; do
  timeout -k 10 120 python tools/passtime.py --dims 1024,1024 --rhs $r --op K 2>/dev/null || exit 1
done | tee gpurun_out/c2_rounds_m.txt
