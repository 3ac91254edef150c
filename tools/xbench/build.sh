#!/bin/bash
# Build xbench variants here (CPU); binaries travel to the GPU box with the
# tree.  Usage: build.sh name:"-DKSTEPS=20 ..." ...
set -e
cd "$(dirname "$0")"
R=../..
mkdir -p bin
FL="-O3 -std=c++17 -ffp-contract=off -fno-fast-math --offload-arch=gfx950 -fno-slp-vectorize -I$R/include -I$R/smi_amd/csrc"
pids=()
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  ( /opt/rocm/bin/hipcc $FL $flags -DVARIANT_NAME="\"$name\"" -Rpass-analysis=kernel-resource-usage \
      xbench.hip -o bin/xbench_$name 2> bin/$name.remarks && \
    grep -E "VGPRs:|Spill|Occupancy|LDS" bin/$name.remarks | sed "s/^/$name: /" ) &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
