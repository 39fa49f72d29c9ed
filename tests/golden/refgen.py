"""The reference's synthetic cluster generator, restated seeded (test fixture).

kano_py/tests/generate.py:5-96 (`ConfigFiles`) draws, with Python's global
`random` and no seed:

  pods      (generatePods, :25-37): pod i is Container("pod<i>", labels) with
            labels["User"] = choice(users) and then randint(0, podLL-1) draws of
            labels[choice(keys)] = choice(values) (a repeated key overwrites);
  policies  (generateConfigFiles, :53-81): per policy, sample(containers, 2);
            the podSelector prints candidates[0]'s labels, a choice of
            "  ingress" / "  egress" sets policyTypes and the rule, and the
            rule's single podSelector peer prints candidates[1]'s labels;
            printLabels (:83-93) writes "User: <value>" then at most three
            other labels in dict order.

This module replays the same draws in the same order from a private
`random.Random(seed)`, so a seeded run equals the reference's generator
after `random.seed(seed)` (make_golden.py checks exactly that against the
reference's own ConfigFiles under py3.9 and stores the digest).  It is pure
Python (runs under the reference's py3.9 and the repo's py3.10).  Only the
parameters the reference uses are kept (podN, policyN, podLL, keyL, valueL,
userL); the file layout is `policy<i>.yml`.
"""
import hashlib
import random

KEYS_DEFAULT = dict(podN=100, policyN=50, podLL=5, keyL=5, valueL=10, userL=5)


class RefGen:
    def __init__(self, seed, podN=100, policyN=50, podLL=5, keyL=5, valueL=10, userL=5):
        self.rng = random.Random(seed)
        self.podN, self.policyN, self.podLL = podN, policyN, podLL
        self.keys = ["key" + str(i) for i in range(keyL)]
        self.values = ["value" + str(i) for i in range(valueL)]
        self.users = ["user" + str(i) for i in range(userL)]
        self.pods = self._pods()              # [(name, labels)]
        self.policies = {}                    # file name -> (select, allow, direction)
        self.files = self._policy_files()     # [(file name, yaml text)]

    # generate.py:25-37
    def _pods(self):
        r = self.rng
        out = []
        for i in range(self.podN):
            labels = {"User": r.choice(self.users)}
            for _ in range(r.randint(0, self.podLL - 1)):
                labels[r.choice(self.keys)] = r.choice(self.values)
            out.append(("pod" + str(i), labels))
        return out

    # generate.py:83-93
    @staticmethod
    def _printed(labels):
        """The dict that printLabels' YAML lines load back as (string values)."""
        d = {"User": str(labels.get("User", ""))}
        for k, v in labels.items():
            if len(d) > 3:
                break
            if k != "User":
                d[str(k)] = str(v)
        return d

    @staticmethod
    def _print_labels(labels, indent):
        s = indent + "User: " + str(labels.get("User", "")) + "\n"
        count = 0
        for k, v in labels.items():
            if count >= 3:
                break
            if k == "User":
                continue
            s += indent + str(k) + ": " + str(v) + "\n"
            count += 1
        return s

    # generate.py:53-81
    def _policy_files(self):
        r = self.rng
        out = []
        for i in range(self.policyN):
            data = ("apiVersion: networking.k8s.io/v1\nkind: NetworkPolicy\nmetadata:\n"
                    "  name: test-network-policy\n  namespace: default\n")
            data += "spec:\n  podSelector:\n    matchLabels:\n"
            a, b = r.sample(range(len(self.pods)), 2)
            data += self._print_labels(self.pods[a][1], "      ")
            data += "  policyTypes:\n"
            ingress = r.choice(["  ingress", "  egress"]) == "  ingress"
            if ingress:
                data += "  - Ingress\n  ingress:\n  - from:\n"
            else:
                data += "  - Egress\n  egress:\n  - to:\n"
            self.policies["policy" + str(i) + ".yml"] = (
                self._printed(self.pods[a][1]), self._printed(self.pods[b][1]),
                "ingress" if ingress else "egress")
            data += "    - podSelector:\n        matchLabels:\n"
            data += self._print_labels(self.pods[b][1], "          ")
            out.append(("policy" + str(i) + ".yml", data))
        return out

    def digest(self) -> str:
        h = hashlib.sha256()
        for name, labels in self.pods:
            h.update(repr((name, sorted(labels.items()))).encode())
        for name, text in self.files:
            h.update(name.encode())
            h.update(text.encode())
        return h.hexdigest()

    def write(self, directory) -> None:
        import os
        os.makedirs(directory, exist_ok=True)
        for name, text in self.files:
            with open(os.path.join(directory, name), "w") as f:
                f.write(text)


def cluster_json(seed, podN, policyN, walk_order):
    """The generated cluster as the oracle's JSON input: pods in order,
    policies in the order kano_py's directory walk parsed their files."""
    g = RefGen(seed, podN=podN, policyN=policyN)
    pols = []
    for f in walk_order:
        sel, alw, d = g.policies[f]
        pols.append({"name": "test-network-policy-" + d, "select": sel, "allow": alw,
                     "direction": d})
    return {"pods": [{"name": nm, "labels": lab} for nm, lab in g.pods], "policies": pols}
