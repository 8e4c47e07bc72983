import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import kyverno_amd as K
from tests.policies import pss_policy, restricted_latest
pol = restricted_latest() if os.environ.get("C2") else pss_policy("golden", "baseline", "latest")
pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p"}, "spec": {"containers": [{"name": "c", "image": "x"}]}}
eng = K.Engine(ordinal=0)
v, _, _ = eng.evaluate(K.PolicySet([pol]), K.Corpus(json.dumps(pod).encode()))
print(v)
