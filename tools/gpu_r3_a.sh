# round 3 GPU call A: fp64 raw-buffer fix check, then the GPU test suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HGP_LIB=$PWD/hipgp_amd/libhipgp_buf64.so timeout -k 10 300 python -u tools/diag_buf64.py 2048x8 1025x8 4096x8 > gpurun_out/diag_buf64_fixed.txt 2>&1 || exit 1
cat gpurun_out/diag_buf64_fixed.txt
LIBS="libhipgp_buf64" REPEAT=1 SHAPES="1025x8 2048x8 4096x8" timeout -k 10 300 bash tools/diag_ab.sh > gpurun_out/diag_contig_fixed.txt 2>&1 || exit 1
cat gpurun_out/diag_contig_fixed.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_a.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu_a.log
exit $rc
