# round 4 GPU call D: row-pass phase stagger variants (K op at C4 / C3); SQ counters of the R^T
# passes at C4 and C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base s2 s4; do
  lib=$PWD/hipgp_amd/libhipgp.so; [ $v = base ] || lib=$PWD/hipgp_amd/libhipgp_$v.so
  for cfg in "4096,4096 25" "2048,2048 200"; do
    set -- $cfg
    echo "variant $v"
    HGP_LIB=$lib timeout -k 10 120 python tools/passtime.py --dims $1 --rhs $2 --op K || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/stagger_d.txt || exit 1
SHAPE=4096,4096 RHS=25 TAG=C4RT OP=RT timeout -k 10 600 bash tools/pmc_sq_cfg.sh > gpurun_out/pmc_sq_C4RT.log 2>&1 || { tail -5 gpurun_out/pmc_sq_C4RT.log; exit 1; }
SHAPE=256,256,128 RHS=25 TAG=C5RT OP=RT timeout -k 10 600 bash tools/pmc_sq_cfg.sh > gpurun_out/pmc_sq_C5RT.log 2>&1 || { tail -5 gpurun_out/pmc_sq_C5RT.log; exit 1; }
SHAPE=4096,4096 RHS=25 TAG=C4K OP=K timeout -k 10 600 bash tools/pmc_sq_cfg.sh > gpurun_out/pmc_sq_C4K.log 2>&1 || { tail -5 gpurun_out/pmc_sq_C4K.log; exit 1; }
echo done
