# round 3 GPU call G: library variants at C4 (and C2): grouped 4096-point rows (g2: G = 2, 4 pairs x
# 2 columns = 128-B segments), running-product stage twiddles (ch), sequential transforms on
# multi-wave lines (sq); per pass K and C^-1, PMC bytes per kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS=${LIBS:-"libhipgp libhipgp_g2 libhipgp_g2c2 libhipgp_g2sq libhipgp_sq libhipgp_ch"}
PMCLIBS=${PMCLIBS:-"libhipgp libhipgp_g2 libhipgp_g2c2 libhipgp_sq"}
for lib in $LIBS; do
  for cfg in ${CFGS:-4096,4096:25:K 4096,4096:25:CINV 1024,1024:32:K 2048,2048:32:K}; do
    d=${cfg%%:*}; rest=${cfg#*:}; r=${rest%%:*}; op=${rest#*:}
    HGP_LIB=$PWD/hipgp_amd/$lib.so timeout -k 10 120 python tools/passtime.py --dims $d --rhs $r --op $op | sed "s/^/$lib /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_${TAG:-g}_passtime.txt || exit 1
# C5 R^T: workspace budget (RHS per chunk) and stream count
[ -n "$NO_RT" ] || for env in "X=0" "HGP_WS_MB=12288" "HGP_WS_MB=26000" "HGP_STREAMS=1" "HGP_WS_MB=26000 HGP_STREAMS=1"; do
  env $env timeout -k 10 120 python tools/passtime.py --dims 256,256,128 --rhs 25 --op RT | sed "s/^/$env /" || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3_g_rt_ws.txt || exit 1
for lib in $PMCLIBS; do
  HGP_LIB=$PWD/hipgp_amd/$lib.so SHAPE=4096,4096 RHS=25 TAG=C4_$lib timeout -k 10 600 bash tools/prof_cfg.sh || exit 1
done
