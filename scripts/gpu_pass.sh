#!/bin/bash
# One GPU pass, parameterised: scripts/gpu_pass.sh <tag> <step>...
# Output under gpurun_out/<tag>/ (copied into profiles/<tag>/ afterwards for the record). Every step
# runs under its own time limit; the pass stops at the first failing step.
#   smoke                 __graft_entry__.smoke()
#   tests[:<pytest -k>]   the -m gpu suite (or the tests matching the -k expression), one process
#   bench:<cfg>[:<args>]  bench.py --config <cfg> <args> (args: comma-separated) -> bench_<cfg>.json
#   trace:<cfg>[:<args>]  rocprofv3 --kernel-trace --stats of that bench run
#   pmc:<cfg>:<counters>[:<args>]  one rocprofv3 --pmc pass (counters comma-separated; one block's
#                         limits per pass, MI355X_MICROARCH.md)
#   traffic:<cfg>:<kernel prefix>[:<args>]  FETCH_SIZE and WRITE_SIZE passes summarised into
#                         gpurun_out/<tag>/pmc_traffic_<cfg>.json (scripts/pmc_summary.py; copy it to perf/)
#   ranks:<n>[:<args>]    bench.py --gpus <n> with gloo collectives (several ranks on one device)
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p "$O"
run() {  # run <name> <timeout> <cmd...>
  local name=$1 to=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n "${TAILN:-3}" "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for st in "$@"; do
  IFS=: read -r kind a1 a2 a3 <<< "$st"
  case $kind in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    tests)
      if [ -n "$a1" ]; then
        TAILN=6 run "tests_$(echo "$a1" | tr -c 'a-zA-Z0-9_' _)" 900 python -u -m pytest tests -m gpu -x -v -k "$a1" --timeout 300 --timeout-method thread
      else
        TAILN=6 run tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
      fi ;;
    bench)
      run "bench_$a1" 400 python bench.py --config "$a1" ${a2//,/ }
      grep '^{' "$O/bench_$a1.log" > "$O/bench_$a1.json" ;;
    trace)
      x=${a2:---steps,20,--warmup,3,--cpu-sample,0}
      run "trace_$a1" 400 rocprofv3 --kernel-trace --stats -d "$O/prof_$a1" -o "$a1" --output-format csv -- \
        python3 bench.py --config "$a1" ${x//,/ } ;;
    pmc)
      x=${a3:---steps,5,--warmup,1,--cpu-sample,0}
      nm=$(echo "$a2" | tr ',' '_' | cut -c1-40)
      run "pmc_${a1}_$nm" 120 rocprofv3 --pmc ${a2//,/ } -d "$O/pmc_$a1" -o "pmc_$nm" --output-format csv -- \
        python3 bench.py --config "$a1" ${x//,/ } ;;
    traffic)
      x=${a3:---steps,20,--warmup,3,--cpu-sample,0,--replicas,20}
      for k in FETCH_SIZE WRITE_SIZE; do
        run "traffic_${a1}_$k" 120 rocprofv3 --pmc $k -d "$O/traffic_$a1" -o "$k" --output-format csv -- \
          python3 bench.py --config "$a1" ${x//,/ }
      done
      run "traffic_${a1}_summary" 60 python3 scripts/pmc_summary.py --dir "$O/traffic_$a1" --kernel "$a2" \
        --out "$O/pmc_traffic_$a1.json" --bench-log "$O/traffic_${a1}_WRITE_SIZE.log" ;;  # copy into perf/ (bench.py reads it there) after the call
    ranks)
      KPE_DIST_BACKEND=gloo run "ranks_$a1" 400 python bench.py --gpus "$a1" ${a2//,/ }
      grep '^{' "$O/ranks_$a1.log" > "$O/ranks_$a1.json" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
exit 0
