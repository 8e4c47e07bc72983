#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of the pattern kernel on C3 / C5 -> perf/pmc_traffic_<cfg>.json
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${CFGS:-c5 c3}; do
  for k in fetch write; do
    K=$(echo $k | tr a-z A-Z)_SIZE
    timeout -s KILL 120 rocprofv3 --pmc $K -d gpurun_out/pt_${c}_$k -o $c --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/pt_${c}_$k.log 2>&1 || exit $?
  done
  python3 scripts/pmc_pattern_traffic.py $c ${KPREFIX:-kpe_pattern_kernel} || exit $?
done
