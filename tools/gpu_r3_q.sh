# round 3 evidence on the final tree (after the tri-row grouping): GPU tests, smoke, bench line,
# rocprofv3 kernel stats of the bench, configs table, compute_kn phases, C4 / C5 R^T passes, and a
# 2-rank same-device (gloo) rehearsal of the multi-rank bench path.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_q.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_q.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_q.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_q.log 2>&1 || { tail -20 gpurun_out/smoke_q.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { tail -20 gpurun_out/bench_q.err; exit 1; }
tail -1 gpurun_out/bench_q.json
bash tools/profile.sh q || exit 1
timeout -k 10 900 python tools/bench_configs.py > gpurun_out/configs_q.jsonl 2> gpurun_out/configs_q.err || { tail -5 gpurun_out/configs_q.err; exit 1; }
timeout -k 10 600 python tools/kn_phases.py --only C5,C4,C3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/kn_phases_q.jsonl || exit 1
for cfg in 256,256,128 4096,4096; do
  timeout -k 10 120 python tools/passtime.py --dims $cfg --rhs 25 --op RT || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/rt_passtime_q.txt || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo --same-device --no-cpu-baseline > gpurun_out/bench_2rank_q.jsonl 2> gpurun_out/bench_2rank_q.err || { tail -10 gpurun_out/bench_2rank_q.err; exit 1; }
tail -1 gpurun_out/bench_2rank_q.jsonl
