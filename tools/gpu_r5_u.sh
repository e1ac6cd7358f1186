# round 5 GPU call U: is the 4096-point column pass's time data dependent?  C4 K and C^-1 op /
# pass times at three kernel lengthscales (the C^-1 conv ran 12 % longer than K's at ell 0.1).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for ell in 0.1 0.01 1.0; do
  for op in K CINV; do
    timeout -k 10 180 python tools/passtime.py --dims 4096,4096 --rhs 25 --op $op --ell $ell 2>/dev/null | sed "s/^/ell$ell /" || exit 1
  done
done | tee gpurun_out/r5u_ell.txt
