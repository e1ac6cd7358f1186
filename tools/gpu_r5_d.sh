# round 5 GPU call D: the chained 2-D PCG iteration (K p -> EPI_RF -> C^-1 r per RHS chunk) and the
# quad layout with tri lines back to one per block: PCG / break-rule / parity tests first, then
# the full suite, then compute_kn phases with the chain on and off, and the per-pass op times.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pcg_break_gpu.py \
  tests/test_cg_gpu.py tests/test_large_gpu.py tests/test_parity_gpu.py > gpurun_out/r5d_pcg.log 2>&1 || { tail -40 gpurun_out/r5d_pcg.log; exit 1; }
tail -1 gpurun_out/r5d_pcg.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread --deselect tests/test_fit_c3_gpu.py::test_c3_settings_fine_diverges_like_reference_fp64 > gpurun_out/r5d_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5d_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r5d_pytest_gpu.log
for c in 1 0; do
  HGP_CHAIN_PCG=$c timeout -k 10 400 python tools/kn_phases.py --only C2,C3,C4 2>/dev/null | sed "s/^/chain$c /" || exit 1
done | tee gpurun_out/r5d_kn_phases.txt
for cfg in "4096,4096 25 K" "4096,4096 25 RT" "1024,1024 32 K"; do
  set -- $cfg
  timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op $3 2>/dev/null || exit 1
done | tee gpurun_out/r5d_passtime.txt
