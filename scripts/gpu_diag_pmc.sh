#!/bin/bash
# VALU / SALU / LDS instruction counts of the scan kernel per diagnostic build (-DKPE_DIAG=N).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in kyverno_amd/libkpe.so kyverno_amd/build/diag/libkpe_d${VARIANTS:-[2468]}.so; do
  tag=$(basename $lib .so)
  KPE_LIB=$PWD/$lib N=1000000 STEPS=20 timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/dp_$tag -o $tag --output-format csv -- python3 scripts/diag_time.py > gpurun_out/dp_$tag.log 2>&1
  rc=$?; echo "== $tag rc=$rc"; grep '^{' gpurun_out/dp_$tag.log
  [ $rc -ge 124 ] && exit $rc
done
exit 0
