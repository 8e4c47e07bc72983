import sys, os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time, kyverno_amd as K
eng = K.Engine(ordinal=0)
nd = K.synth_resources(0xC2, 1000000, mix=K.SYNTH_PODS)
for k in range(4):
    t = time.perf_counter(); c = K.Corpus(nd, docs=False); t1 = time.perf_counter()
    c.upload(eng.device); t2 = time.perf_counter()
    print(f"flatten {t1-t:.3f} upload {t2-t1:.3f}", flush=True)
