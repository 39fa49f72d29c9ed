"""Add policy_shadow's pair count from the C/numpy oracle to the big-config
goldens (run after make_golden.py --big; repo python3):

    python3 tests/golden/oracle_counts.py C3 C4

kano_py cannot materialise C4's ~1e11 pairs, so C4's count comes from
oracle.kano_oracle.shadow_count_grouped (pinned against kano_py's own counts
on every other golden, tests/test_oracle_golden.py); on C3 both exist and
must agree."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kubernetes-verification_amd"))

from kano.synth import make_config  # noqa: E402
from oracle import kano_oracle as orc  # noqa: E402


def main():
    for name in sys.argv[1:]:
        path = os.path.join(HERE, "expected", name + ".json")
        with open(path) as f:
            rec = json.load(f)
        cl = make_config(name)
        assert cl.fingerprint() == rec["seed"]["fingerprint"]
        cnt = orc.shadow_count_grouped(cl.to_json_obj())
        sh = rec["policy_shadow"]
        if "count" in sh:
            assert sh["count"] == cnt, (name, sh["count"], cnt)
        sh["oracle_count"] = cnt
        with open(path, "w") as f:
            json.dump(rec, f, separators=(",", ":"))
        print(name, "oracle shadow count", cnt)


if __name__ == "__main__":
    main()
