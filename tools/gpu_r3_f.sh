# round 3 GPU call F: after the straight-line fold loads (row / line / pass kernels): GPU tests,
# the bench line, per-pass times C2 / C3 / C4 / C5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_f.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu_f.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r3_bench_f.json 2> gpurun_out/r3_bench_f.err || { tail -5 gpurun_out/r3_bench_f.err; exit 1; }
cat gpurun_out/r3_bench_f.json
for dr in 1024,1024:32:K 2048,2048:32:K 4096,4096:25:K 256,256,128:25:K 256,256,128:25:RT; do
  d=${dr%%:*}; rest=${dr#*:}; r=${rest%%:*}; op=${rest#*:}
  timeout -k 10 120 python tools/passtime.py --dims $d --rhs $r --op $op || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_f_passtime.txt || exit 1
exit $rc
