#!/bin/bash
# rocprofv3 kernel durations of the diagnostic LEAN builds (empty / prologue-only / no-PSS / full)
# at two grid sizes. Output: gpurun_out/diag_prof.log
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/diag_prof.log
: > $out
for v in d16 d8 d2 full; do
  for bpc in 7 2; do
    lib=kyverno_amd/build/diag/libkpe_$v.so; [ $v = full ] && lib=kyverno_amd/libkpe.so
    KPE_SCAN_BPC=$bpc KPE_LIB=$PWD/$lib STEPS=30 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof_${v}_$bpc -o p --output-format csv -- python3 scripts/diag_time.py > /dev/null 2>&1 || { echo "$v $bpc failed" >> $out; exit 1; }
    f=$(ls gpurun_out/dprof_${v}_$bpc/*kernel_stats.csv | head -1)
    echo "$v bpc=$bpc $(grep lean_kernel $f | cut -d, -f2-4)" >> $out
  done
done
cat $out
