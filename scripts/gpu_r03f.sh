#!/bin/bash
# Site-kernel variants (KPE_LIB): C5 / C3 kernel traces (per-kernel means) and bench lines.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS:-loop2 loop4}; do
  for c in c5 c3; do
    KPE_LIB=$PWD/kyverno_amd/build/var/libkpe_$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_${c}_$v -o $c --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/tr_${c}_$v.log 2>&1 || exit $?
    f=$(find gpurun_out/tr_${c}_$v -name "*kernel_stats.csv" | head -1); echo "== $c $v"; cut -d, -f1-4 "$f" | grep -E "site|pattern|cond"
  done
done
