# round 3 GPU call O: C2 column-pass occupancy variants (c2m3: 256-thread blocks at 3 waves/SIMD;
# c2t4: 256-thread blocks at 4) against the default, bench lines; C4 R^T / C^-1 / K passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libhipgp libhipgp_c2m3 libhipgp_c2t4 libhipgp; do
  HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 300 python bench.py --no-cpu-baseline --pcg-reps 3 > gpurun_out/o_$lib.json 2> gpurun_out/o_$lib.err || { tail -5 gpurun_out/o_$lib.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/o_$lib.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$lib', round(d['value']), round(r['frac'],4), round(d['pcg_wall_clock_ms'],2), [p['ms'] for p in r['passes']])"
done 2>&1 | tee gpurun_out/r3_o_c2.txt || exit 1
for op in RT CINV K; do
  timeout -k 10 120 python tools/passtime.py --dims 4096,4096 --rhs 25 --op $op || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_o_c4.txt || exit 1
