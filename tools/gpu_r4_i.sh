# round 4 GPU call I: one vs two RHS streams for the 2-D / 3-D operators at C3 / C4 / C5 (op times,
# compute_kn phases); the drop-in long-axis compute_kn test
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_long_axis_gpu.py -q --timeout 300 --timeout-method thread -k drop_in > gpurun_out/pytest_i.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_i.log; [ $rc -le 1 ] || exit 1
for ns in 2 1; do
  for cfg in "2048,2048 200" "4096,4096 25" "256,256,128 25"; do
    set -- $cfg
    echo "streams $ns"
    HGP_STREAMS=$ns timeout -k 10 120 python tools/passtime.py --dims $1 --rhs $2 --op K || exit 1
    HGP_STREAMS=$ns timeout -k 10 120 python tools/passtime.py --dims $1 --rhs $2 --op RT || exit 1
  done
  HGP_STREAMS=$ns timeout -k 10 600 python tools/kn_phases.py --only C3,C4,C5 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/streams_i.txt || exit 1
