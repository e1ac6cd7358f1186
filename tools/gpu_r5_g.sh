# round 5 GPU call G: packed DC / Nyquist columns of the 2-D K / C^-1 intermediate (PassDesc::dcny):
# the GPU suite (fp32 and fp64 2-D parity through the packed path), then HGP_DCNY=1 vs 0 on the
# C2 op (per-pass), the bench line and C2 compute_kn, twice each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r5g_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5g_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r5g_pytest_gpu.log
for r in 1 2; do
  for dn in 1 0; do
    HGP_DCNY=$dn timeout -k 10 120 python tools/passtime.py --dims 1024,1024 --rhs 32 --op K 2>/dev/null | sed "s/^/dcny$dn /" || exit 1
    HGP_DCNY=$dn timeout -k 10 300 python bench.py --no-cpu-baseline --no-c4-leg > gpurun_out/r5g_bench_$dn.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/r5g_bench_$dn.json').read().strip().splitlines()[-1]); print('dcny$dn bench', round(d['value']), round(d['roofline']['frac'],3), 'pcg', round(d['pcg_wall_clock_ms'],2), [(p['ms'], p['frac']) for p in d['roofline']['passes']])"
  done
done | tee gpurun_out/r5g_dcny.txt
