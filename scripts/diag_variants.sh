#!/bin/bash
# Time the scan kernel of every diagnostic / register-budget build (make -C kyverno_amd diag waves) on C2.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
KPE_DEBUG=1 KPE_LIB=$PWD/kyverno_amd/libkpe.so N=1000000 STEPS=2 timeout 120 python3 scripts/diag_time.py 2>&1 | grep -v "^{" | head -4
for lib in kyverno_amd/libkpe.so kyverno_amd/build/diag/libkpe_${VARIANTS:-[dw]}*.so; do
  KPE_LIB=$PWD/$lib timeout -k 10 180 python3 scripts/diag_time.py >> gpurun_out/diag.jsonl 2> gpurun_out/diag_err.log
  rc=$?; [ $rc -ne 0 ] && { echo "$lib rc=$rc"; tail -5 gpurun_out/diag_err.log; exit $rc; }
done
cat gpurun_out/diag.jsonl
