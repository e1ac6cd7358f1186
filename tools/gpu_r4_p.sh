# round 4 GPU call P: clamped-case PCG divergence diagnostic (tools/clamp_diag.py) for G4b / G7 fp64.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in G4b G7 G4c; do
  echo "== $c"; timeout -k 10 120 python tools/clamp_diag.py $c f64 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/clamp_diag_p.txt
