#!/bin/bash
# A/B of the C2 LEAN scan variants (kpe_lean5<1> / <2>, kpe_lean4, kpe_lean3) through bench.py;
# one JSON line per variant under gpurun_out/lean_ab/.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/lean_ab
for v in lean5 lean5_t2 lean4 lean3; do
  case $v in
    lean5) envs="" ;;
    lean5_t2) envs="KPE_LEAN5_T2=1" ;;
    lean4) envs="KPE_LEAN4=1" ;;
    lean3) envs="KPE_LEAN3=1" ;;
  esac
  echo "== $v ($(date +%T))"
  env $envs timeout -k 10 300 python bench.py --cpu-sample 0 --steps 200 --warmup 20 > gpurun_out/lean_ab/$v.json 2> gpurun_out/lean_ab/$v.err
  rc=$?
  echo "== $v rc=$rc"
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
try:
    d = json.load(open(f"gpurun_out/lean_ab/{v}.json"))
    r = d["roofline"]
    print(v, "value %.3e" % d["value"], "step %.2f us" % (d["ms_per_step"] * 1e3), "kernel %.2f us" % (r["kernel_ms"] * 1e3),
          "bytes %.1f MB" % (r["alg_bytes_per_launch"] / 1e6), "frac %.3f" % r["frac"],
          "masks %.2f us" % (d["masks_step"]["scan_kernel_ms"] * 1e3))
except Exception as e:
    print(v, "no result", e)
PY
  if [ $rc -ge 124 ]; then exit $rc; fi
done
