# round 4 GPU call J: packed-fp32 FFT arithmetic (HGP_PK32=1 build, libhipgp_pk.so) -- parity of the
# fp32 operators and PCG against the oracle / fp64, then per-pass times A/B against the shipped build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
PK=$PWD/hipgp_amd/libhipgp_pk.so
HGP_LIB=$PK timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_large_gpu.py tests/test_pcg_break_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_j.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_j.log; [ $rc -eq 0 ] || exit 1
for lib in base pk; do
  if [ $lib = pk ]; then export HGP_LIB=$PK; else unset HGP_LIB; fi
  for cfg in "1024,1024 32" "4096,4096 25" "2048,2048 200" "256,256,128 25"; do
    set -- $cfg
    for op in K RT; do
      echo -n "$lib "; timeout -k 10 120 python tools/passtime.py --dims $1 --rhs $2 --op $op || exit 1
    done
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/pk_j.txt || exit 1
for lib in base pk; do
  if [ $lib = pk ]; then export HGP_LIB=$PK; else unset HGP_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs > gpurun_out/bench_j_$lib.json 2> gpurun_out/bench_j_$lib.err || { tail -20 gpurun_out/bench_j_$lib.err; exit 1; }
  echo -n "$lib "; tail -1 gpurun_out/bench_j_$lib.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['pcg_wall_clock_ms'], d['roofline']['frac'])"
done
