# round 3 GPU call I: after the long-line column-pass geometry (1-line blocks, 3 waves/SIMD at 4096):
# GPU tests, per-pass times C2-C4 with the stream count / workspace budget varied, the bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_i.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu_i.log
[ $rc -le 1 ] || exit $rc
for env in "X=0" "HGP_STREAMS=1" "HGP_WS_MB=4096" "HGP_WS_MB=4096 HGP_STREAMS=1"; do
  for cfg in 4096,4096:25:K 2048,2048:32:K 2048,2048:200:K 1024,1024:32:K; do
    d=${cfg%%:*}; rest=${cfg#*:}; r=${rest%%:*}; op=${rest#*:}
    env $env timeout -k 10 120 python tools/passtime.py --dims $d --rhs $r --op $op | sed "s/^/$env /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_i_passtime.txt || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r3_bench_i.json 2> gpurun_out/r3_bench_i.err || { tail -5 gpurun_out/r3_bench_i.err; exit 1; }
cat gpurun_out/r3_bench_i.json
exit $rc
