# A/B of compile-time occupancy knobs (diag builds: make -C kyverno_amd var NAME=... DEFS=...)
run() {  # run <tag> <lib> <config> <steps>
  KPE_LIB=$2 timeout -k 10 400 python bench.py --config $3 --steps $4 --cpu-sample 0 > gpurun_out/ab_$1.log 2>&1 || exit 1
  tail -1 gpurun_out/ab_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1', d['value'], d['ms_per_step'], r['kernel_ms'])"
}
D=kyverno_amd/build/diag
run c3_base kyverno_amd/libkpe.so c3 20
run c3_pw6 $D/libkpe_pw6.so c3 20
run c3_pw7 $D/libkpe_pw7.so c3 20
run c5_pw7 $D/libkpe_pw7.so c5 20
