set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 ./tools/buf_semantics > gpurun_out/buf_semantics.txt 2>&1 && cat gpurun_out/buf_semantics.txt &&
HGP_LIB=$PWD/hipgp_amd/libhipgp_buf64.so timeout -k 10 300 python -u tools/diag_buf64.py 2048x8 1025x8 4096x8 > gpurun_out/diag_buf64.txt 2>&1; rc=$?; cat gpurun_out/diag_buf64.txt; exit $rc
