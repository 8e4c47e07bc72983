#!/bin/bash
# One GPU session: scan-kernel phase costs (diagnostic builds, VARIANTS), then rocprofv3 kernel
# traces of the C2 bench and of the C3 / C5 pattern-kernel benches (gpurun_out/prof_<cfg>).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$VARIANTS" ]; then
  bash scripts/diag_variants.sh || exit $?
fi
for cfg in ${CONFIGS:-c2 c3 c5}; do
  args="--config $cfg --cpu-sample 0"
  [ "$cfg" = c2 ] && args="$args --steps 100 --warmup 10" || args="$args --steps 10 --warmup 2"
  echo "== trace $cfg"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$cfg -o $cfg --output-format csv \
    -- python3 bench.py $args > gpurun_out/prof_$cfg.log 2>&1
  rc=$?; echo "rc=$rc"; tail -c 600 gpurun_out/prof_$cfg.log; echo
  [ $rc -ne 0 ] && exit $rc
done
exit 0
