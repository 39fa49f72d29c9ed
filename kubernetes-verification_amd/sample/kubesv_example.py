"""kubesv's sample cluster (kubesv/sample/example.py:106-174, ``paper_example``)
for kano.k8s: two namespaces, twelve pods (role x namespace x env) and one
NetworkPolicy in "default" that selects role NotIn [tomcat, nginx], admits
ingress from tomcat pods of namespaces labelled nonsense=default and sends
egress to non-db, non-nginx pods of namespaces without the label "l"
(the operator is spelled ``DoesNotExists`` there, which kubesv reads)."""
from itertools import product

from kano import k8s

POLICY = """
apiVersion: v1
kind: NetworkPolicy
metadata:
  name: allow-default-nginx
  namespace: default
spec:
  podSelector:
    matchExpressions:
      - {key: role, operator: NotIn, values: [tomcat, nginx]}
  policyTypes: [Ingress, Egress]
  ingress:
  - from:
    - namespaceSelector:
        matchLabels: {nonsense: default}
      podSelector:
        matchLabels: {role: tomcat}
    ports:
    - {protocol: TCP, port: 6379}
  egress:
  - to:
    - podSelector:
        matchExpressions:
          - {key: role, operator: NotIn, values: [db, nginx]}
      namespaceSelector:
        matchExpressions:
          - {key: l, operator: DoesNotExists}
    ports:
    - {protocol: TCP, port: 5978}
"""


def paper_example():
    nams = [k8s.Namespace("default", {"nonsense": "default"}),
            k8s.Namespace("minikube", {"nonsense": "emmm", "l": "minikube"})]
    pods = [k8s.Pod(f"{role}_{i}", ns, {"env": env, "role": role})
            for i, (role, ns, env) in enumerate(product(["db", "nginx", "tomcat"],
                                                        ["default", "minikube"],
                                                        ["prod", "test"]))]
    pols = [k8s.from_yaml("V1NetworkPolicy", POLICY)]
    return pods, pols, nams
