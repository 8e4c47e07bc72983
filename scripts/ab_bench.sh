#!/bin/bash
# A/B bench lines of one config under several environments (library variants, knobs), each run
# under its own time limit; outputs gpurun_out/<tag>/ab_<cfg>_<name>.json.
# Usage: scripts/ab_bench.sh <tag> <cfg> <name>=<ENV=VAL[,ENV=VAL]>|<name>=- ...
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=$1 CFG=$2
shift 2
O=gpurun_out/$TAG
mkdir -p "$O"
for spec in "$@"; do
  name=${spec%%=*} envs=${spec#*=}
  args=()
  [ "$envs" != "-" ] && IFS=, read -ra args <<< "$envs"
  echo "== $CFG $name ($(date +%T)) ${args[*]}"
  env "${args[@]}" timeout -k 10 300 python bench.py --config "$CFG" --steps 20 --warmup 5 --cpu-sample 0 \
    > "$O/ab_${CFG}_$name.log" 2>&1
  rc=$?
  echo "== rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$O/ab_${CFG}_$name.log"; exit $rc; }
  grep '^{' "$O/ab_${CFG}_$name.log" > "$O/ab_${CFG}_$name.json"
  python3 -c "import json,sys; d=json.load(open('$O/ab_${CFG}_$name.json')); r=d['roofline']; print('$name', round(d['ms_per_step'],4), 'ms/step', round(r['kernel_ms'],4), 'ms kernel', round(r['frac'],3))"
done
