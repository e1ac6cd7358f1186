# round 5 GPU call C: the quad-order G = 4 intermediate (LAY_CONTIG_Q): GPU suite, then per-pass
# times of C4 K / C^-1 / R^T, C3 K, C2 K and per-kernel PMC bytes of C4 K and C4 R^T.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread \
  tests/test_fit_sharded_gpu.py "tests/test_large_gpu.py::test_configs_own_batch_B200" \
  "tests/test_slab_gpu.py::test_slab_C5_geometry" > gpurun_out/r5c_new.log 2>&1 || { tail -40 gpurun_out/r5c_new.log; exit 1; }
grep -E "PASSED|FAILED|rel err|rel diff" gpurun_out/r5c_new.log | tail -40
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread --deselect tests/test_fit_c3_gpu.py::test_c3_settings_fine_diverges_like_reference_fp64 > gpurun_out/r5c_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5c_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r5c_pytest_gpu.log
for cfg in "4096,4096 25 K" "4096,4096 25 CINV" "4096,4096 25 RT" "2048,2048 200 K" "1024,1024 32 K"; do
  set -- $cfg
  timeout -k 10 180 python tools/passtime.py --dims $1 --rhs $2 --op $3 2>/dev/null || exit 1
done | tee gpurun_out/r5c_passtime.txt
SHAPE=4096,4096 RHS=25 TAG=C4K OP=K bash tools/prof_cfg.sh > gpurun_out/r5c_C4K_bytes.txt 2>&1 || { tail -5 gpurun_out/r5c_C4K_bytes.txt; exit 1; }
SHAPE=4096,4096 RHS=25 TAG=C4RT OP=RT NOPS=4 bash tools/prof_cfg.sh > gpurun_out/r5c_C4RT_bytes.txt 2>&1 || { tail -5 gpurun_out/r5c_C4RT_bytes.txt; exit 1; }
tail -12 gpurun_out/r5c_C4K_bytes.txt gpurun_out/r5c_C4RT_bytes.txt
