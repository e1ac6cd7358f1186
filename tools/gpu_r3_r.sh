# round 3 GPU call R: rocprofv3 kernel stats of compute_kn at C5 and C4 (tools/kn_phases.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in C5 C4; do
  rm -rf gpurun_out/prof_kn_$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kn_$c -o run --output-format csv -- \
    python3 tools/kn_phases.py --only $c > gpurun_out/prof_kn_$c.log 2>&1 || { tail -5 gpurun_out/prof_kn_$c.log; exit 1; }
  f=$(find gpurun_out/prof_kn_$c -name "*kernel_stats.csv" | head -1)
  head -16 "$f" | cut -c1-160
done
