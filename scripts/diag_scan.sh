#!/bin/bash
# Diagnostic variants of the scan side (kernels.hip -DKPE_SCAN_ONLY -DKPE_DIAG=<bits>): the WIDE
# general scan without its rule evaluation (1), term evaluation (2) or label fold (4), linked into
# kyverno_amd/build/var/libkpe_d<bits>.so (in-tree, so gpurun ships them; KPE_LIB selects one).
# Usage: scripts/diag_scan.sh 1 3 7 ...
set -e
cd "$(dirname "$0")/../kyverno_amd"
ROCM=${ROCM:-/opt/rocm}
mkdir -p build/var
for d in "$@"; do
  $ROCM/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -munsafe-fp-atomics -fno-vectorize \
    -fno-slp-vectorize -DKPE_SCAN_ONLY -DKPE_DIAG=$d -c csrc/kernels.hip -o build/var/kernels_scan_d$d.o
  $ROCM/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build/var/libkpe_d$d.so build/flatten.o build/program.o \
    build/synth.o build/pss_msg.o build/rhash.o build/kpe_api.o build/var/kernels_scan_d$d.o build/kernels_vm1.o build/kernels_vm2.o build/kernels_vm3.o -lpthread
  echo "built build/var/libkpe_d$d.so"
done
