# round 4 GPU call L: packed-fp32 products as one asm statement (default; hazard s_nops between
# inline-asm results -31 %) vs two statements (libhipgp_split.so) -- parity subset on the default,
# per-pass times A/B at C2 / C4 / C3 / C5, bench line A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_large_gpu.py tests/test_pcg_break_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_l.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_l.log; [ $rc -eq 0 ] || exit 1
for lib in one split one split; do
  if [ $lib = split ]; then export HGP_LIB=$PWD/hipgp_amd/libhipgp_split.so; else unset HGP_LIB; fi
  for cfg in "1024,1024 32" "4096,4096 25" "2048,2048 200" "256,256,128 25"; do
    set -- $cfg
    for op in K RT; do
      timeout -k 10 120 python tools/passtime.py --dims $1 --rhs $2 --op $op 2>/dev/null | sed "s/^/$lib /" || exit 1
    done
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/split_l.txt || exit 1
for lib in one split one split; do
  if [ $lib = split ]; then export HGP_LIB=$PWD/hipgp_amd/libhipgp_split.so; else unset HGP_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs > gpurun_out/bench_l_$lib.json 2> gpurun_out/bench_l_$lib.err || { tail -20 gpurun_out/bench_l_$lib.err; exit 1; }
  echo -n "$lib "; tail -1 gpurun_out/bench_l_$lib.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['pcg_wall_clock_ms'], d['roofline']['frac'])"
done 2>&1 | tee gpurun_out/bench_l.txt
