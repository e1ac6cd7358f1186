# round 4 evidence on the final tree: GPU tests, smoke, the bench line, rocprofv3 kernel stats of
# the bench, PMC HBM bytes of the C2 K matvec, the five-config table, compute_kn phases, C5 ops.
# Each GPU step under its own limit; results under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -2 gpurun_out/smoke_final.log
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
tail -1 gpurun_out/bench_final.json
bash tools/profile.sh final || exit 1
bash tools/pmc_kop.sh > gpurun_out/pmc_kop.log 2>&1 || { tail -20 gpurun_out/pmc_kop.log; exit 1; }
grep traffic_bytes_per_op gpurun_out/pmc_kop/pmc_kop_C2.json
timeout -k 10 900 python tools/bench_configs.py > gpurun_out/configs_final.jsonl 2> gpurun_out/configs_final.err || { tail -5 gpurun_out/configs_final.err; exit 1; }
timeout -k 10 600 python tools/kn_phases.py --only C5,C4,C3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/kn_phases_final.jsonl || exit 1
for op in RT K; do
  timeout -k 10 120 python tools/passtime.py --dims 256,256,128 --rhs 25 --op $op || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/c5_passtime_final.txt || exit 1
