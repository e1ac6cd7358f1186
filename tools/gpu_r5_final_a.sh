# round 5 evidence on the final tree (part A): GPU tests, smoke, the bench line, rocprofv3 kernel
# stats of the bench's headline op alone (--kop-only), PMC HBM bytes of the C2 K matvec.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -2 gpurun_out/smoke_final.log
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
tail -1 gpurun_out/bench_final.json | cut -c1-400
BENCH_ARGS="--kop-only --steps 50 --warmup 5" bash tools/profile.sh kop_final || exit 1
bash tools/pmc_kop.sh > gpurun_out/pmc_kop.log 2>&1 || { tail -20 gpurun_out/pmc_kop.log; exit 1; }
grep traffic_bytes_per_op gpurun_out/pmc_kop/pmc_kop_C2.json | cut -c1-300
