#!/bin/bash
# Register / spill / scratch summary of every kernel in the built code object (gfx950).
set -e
T=$(mktemp -d)
for O in ${1:-kyverno_amd/build/kernels_scan.o kyverno_amd/build/kernels_vm1.o kyverno_amd/build/kernels_vm2.o kyverno_amd/build/kernels_vm3.o}; do
B=/opt/rocm/lib/llvm/bin
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fb.bin "$O"
$B/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$T/fb.bin --output=$T/k.co --unbundle
$B/llvm-readelf --notes $T/k.co | awk '
  /^ +\.name:/ {name=$2}
  /\.private_segment_fixed_size:/ {priv=$2}
  /\.sgpr_spill_count:/ {ss=$2}
  /\.vgpr_count:/ {vc=$2}
  /\.vgpr_spill_count:/ {vs=$2; printf "%-70s vgpr=%-4s vspill=%-4s sspill=%-4s scratch=%s\n", name, vc, vs, ss, priv}'
done
rm -rf $T
