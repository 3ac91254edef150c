#!/bin/bash
# Build the element-channel benchmark against the in-tree library (run on the CPU).
set -e
cd "$(dirname "$0")"
R=$(cd ../.. && pwd)
gcc -O2 -std=gnu11 -I$R/include chanbench.c -o chanbench -L$R/smi_amd/_build -lsmi_amd -Wl,-rpath,'$ORIGIN/../../smi_amd/_build' -lpthread
