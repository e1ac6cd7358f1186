# round 4 GPU call V: grid-stride clamp kernel (one atomic per block of a <= 1024-block sweep) --
# parity subset, then the C2 compute_kn kernel stats again.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_long_axis_gpu.py tests/test_model_gpu.py tests/test_grad_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_v.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_v.log; [ $rc -eq 0 ] || exit 1
OUT=gpurun_out/prof_kn_c2v
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
  python3 tools/kn_phases.py --only C2 > $OUT/kn.log 2>&1 || { tail -5 $OUT/kn.log; exit 1; }
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kn_c2v_kernel_stats.csv
grep -E "k_clamp|Name" gpurun_out/kn_c2v_kernel_stats.csv | cut -c1-160
grep -v amdgpu $OUT/kn.log | grep config
