#!/bin/bash
# Build the sweep microbenchmark variants (run here, on the CPU; the binaries
# travel to the GPU box with the tree).  Usage: build.sh [name:flags ...]
set -e
cd "$(dirname "$0")"
R=../..
mkdir -p bin
FL="-O3 -std=c++17 -ffp-contract=off -fno-fast-math --offload-arch=gfx950 -fno-slp-vectorize -I$R/include -I$R/smi_amd/csrc -I."
if [ $# -eq 0 ]; then set -- "lib:"; fi
pids=()
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc $FL $flags -DVARIANT_NAME="\"$name\"" sweepbench.hip -o bin/sweepbench_$name &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls bin
