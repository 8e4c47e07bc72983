cd $GRAFT_REPO_ROOT
for cfg in "1 kyverno_amd/libkpe.so" "2 kyverno_amd/libkpe.so" "3 kyverno_amd/libkpe.so" "2 kyverno_amd/build/diag/libkpe_w6.so" "3 kyverno_amd/build/diag/libkpe_w6.so"; do
  set -- $cfg
  echo "lanes=$1 lib=$2"
  KPE_LANES=$1 KPE_LIB=$PWD/$2 timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-sample 0 --replicas 8 > gpurun_out/lanes.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/lanes.json'));print(round(d['value']/1e9,1), round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))"
done
