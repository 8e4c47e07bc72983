#!/bin/bash
# Pattern-kernel experiments on C5 / C3 through bench.py: the current build and the diagnostic
# builds without the VM (libkpe_d512.so: the rule loop alone) and with every scalar leaf holding
# without evaluation (libkpe_d1024.so: the walk alone).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pat_ab
for cfg in c5 c3; do
  for v in base novm leafless; do
    lib=""
    [ $v = novm ] && lib="KPE_LIB=kyverno_amd/build/diag/libkpe_d512.so"
    [ $v = leafless ] && lib="KPE_LIB=kyverno_amd/build/diag/libkpe_d1024.so"
    echo "== $cfg $v ($(date +%T))"
    env $lib timeout -k 10 400 python bench.py --config $cfg --cpu-sample 0 --steps 20 --warmup 3 \
      > gpurun_out/pat_ab/${cfg}_$v.json 2> gpurun_out/pat_ab/${cfg}_$v.err
    rc=$?
    echo "== rc=$rc"
    python - "$cfg" "$v" <<'PY'
import json, sys
c, v = sys.argv[1:]
try:
    d = json.load(open(f"gpurun_out/pat_ab/{c}_{v}.json"))
    r = d["roofline"]
    print(c, v, "value %.3e" % d["value"], "step %.3f ms" % d["ms_per_step"], r.get("kernel"), "kernel %.3f ms" % r["kernel_ms"],
          "scan", r.get("scan_kernel"))
except Exception as e:
    print(c, v, "no result", e)
PY
    if [ $rc -ge 124 ]; then exit $rc; fi
  done
done
