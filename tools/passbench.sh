#!/bin/bash
# Build (BUILD=1, here) or run (GPU box) the pass microbenchmark in several block shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARS=(
  "base:-DHGP_CMAX_STRIDED=4 -DHGP_MINW_STRIDED=2 -DHGP_MINW_ROW=2"
#  "cl2:-DHGP_CMAX_STRIDED=4 -DHGP_MINW_STRIDED=2 -DHGP_CONV_LINES=2"
#  "cl8:-DHGP_CMAX_STRIDED=4 -DHGP_MINW_STRIDED=2 -DHGP_CONV_LINES=8"
#  "cl4w3:-DHGP_CMAX_STRIDED=4 -DHGP_MINW_STRIDED=2 -DHGP_CONV_LINES=4 -DHGP_MINW_CONV=3"
)
mkdir -p build gpurun_out
for v in "${VARS[@]}"; do
  name=${v%%:*}; flags=${v#*:}
  if [ -n "$BUILD" ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I hipgp_amd/csrc $flags ${EXTRA:-} tools/passbench.hip -o build/passbench_$name &
  else
    echo "== $name ($flags)"
    for b in build/passbench_${name}*; do echo "-- $b"; timeout -k 5 60 ./$b ${Q:-32} || exit $?; done
  fi
done
wait
