# round 4 GPU call N: the config-4 strong leg (200 RHS at 4096^2) in the bench line -- N = 1, and the
# 2-rank same-device gloo rehearsal (100 RHS per rank).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_n.json 2> gpurun_out/bench_n.err || { tail -20 gpurun_out/bench_n.err; exit 1; }
tail -1 gpurun_out/bench_n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['pcg_wall_clock_ms'], d['strong'], d['elbo_step'], d['strong_c4'])"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --same-device --backend gloo --no-cpu-baseline > gpurun_out/bench_2rank_n.jsonl 2> gpurun_out/bench_2rank_n.err || { tail -20 gpurun_out/bench_2rank_n.err; exit 1; }
tail -1 gpurun_out/bench_2rank_n.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['strong'], d['elbo_step'], d['strong_c4'])"
