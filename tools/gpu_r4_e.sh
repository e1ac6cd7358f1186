# round 4 GPU call E: grouped 4096-point rows re-measured on the spill-free tree (K op at C4);
# PCG chunking at C2 (compute_kn phases under workspace budgets / 3 streams); C2-C5 compute_kn
# phases on this tree; the 2-rank same-device bench rehearsal (gloo) with the strong / ELBO legs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base g2 g4; do
  lib=$PWD/hipgp_amd/libhipgp.so; [ $v = base ] || lib=$PWD/hipgp_amd/libhipgp_$v.so
  echo "variant $v"
  HGP_LIB=$lib timeout -k 10 120 python tools/passtime.py --dims 4096,4096 --rhs 25 --op K || exit 1
  HGP_LIB=$lib timeout -k 10 120 python tools/passtime.py --dims 4096,4096 --rhs 25 --op CINV || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/g4096_e.txt || exit 1
for env in "" "HGP_WS_MB=135" "HGP_WS_MB=270" "HGP_WS_MB=540" "HGP_STREAMS=3"; do
  echo "env: $env"
  env $env timeout -k 10 300 python tools/kn_phases.py --only C2 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/kn_c2_e.txt || exit 1
timeout -k 10 600 python tools/kn_phases.py --only C5,C4,C3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/kn_phases_e.jsonl || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --same-device --backend gloo --no-cpu-baseline > gpurun_out/bench_2rank_e.jsonl 2> gpurun_out/bench_2rank_e.err || { tail -20 gpurun_out/bench_2rank_e.err; exit 1; }
tail -1 gpurun_out/bench_2rank_e.jsonl
HGP_GRAPH=0 timeout -k 10 400 python bench.py --no-cpu-baseline --no-legs > gpurun_out/bench_nograph_e.json 2> gpurun_out/bench_nograph_e.err || { tail -20 gpurun_out/bench_nograph_e.err; exit 1; }
tail -1 gpurun_out/bench_nograph_e.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('no graph', d['value'], d['ms_per_step'], d['roofline']['frac'])"
