# round 5 GPU call B: the new parity / API tests (graph key, configs' own B = 200, slab at C5
# geometry, sharded fit through svigp_fit, slab-sharded compute_kn), then the full GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread \
  tests/test_graph_gpu.py tests/test_fit_sharded_gpu.py "tests/test_large_gpu.py::test_configs_own_batch_B200" \
  "tests/test_slab_gpu.py::test_slab_C5_geometry" > gpurun_out/r5b_new.log 2>&1 || { tail -40 gpurun_out/r5b_new.log; exit 1; }
grep -E "PASSED|FAILED|rel err|rel diff" gpurun_out/r5b_new.log | tail -40
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r5b_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5b_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r5b_pytest_gpu.log
