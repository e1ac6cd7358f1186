# round 4 GPU call U: rocprofv3 kernel stats of compute_kn at C2 alone (kn_phases: set-up + PCG(20) +
# R^T, median of 3 after one warm-up = 4 compute_kn) -- the per-kernel split of the headline PCG
# wall-clock.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/prof_kn_c2
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
  python3 tools/kn_phases.py --only C2 > $OUT/kn.log 2>&1 || { tail -5 $OUT/kn.log; exit 1; }
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kn_c2_kernel_stats.csv
head -16 gpurun_out/kn_c2_kernel_stats.csv | cut -c1-160
grep -v amdgpu $OUT/kn.log | tail -2
