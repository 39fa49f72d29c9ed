"""YAML front-end, drop-in for ``kano.parser`` of kano_py
(kano_py/kano/parser.py:11-101).

Behaviour kept exactly (quirk Q8): one Policy per ingress /
egress *rule*; its allow side is the podSelector of the LAST peer of the rule
that has one (None when no peer has one); ``ports`` of a peer become the
policy's protocol; one Container per ``spec.containers[]`` entry, all sharing
the pod's labels dict (Q9); a file that fails to load or convert prints
"Error opening or reading file <path>"; in directory mode the first bad file
ends the walk ("Error opening or reading directory") keeping what was already
appended; files are visited in ``os.walk`` order.  Values are typed by the
YAML 1.1 resolver of PyYAML (libyaml ``CLoader`` when available), as in the
reference.
"""
from __future__ import annotations

import os

from yaml import load

try:
    from yaml import CLoader as Loader
except ImportError:  # pragma: no cover
    from yaml import Loader

from .model import *  # noqa: F401,F403
from .model import Container, Policy, PolicyAllow, PolicyEgress, PolicyIngress, PolicySelect


def _rule_allow(peers):
    allow, ports = None, None
    for peer in peers:
        if "podSelector" in peer:
            allow = peer["podSelector"]["matchLabels"]
        if "ports" in peer:
            ports = [peer["ports"]["protocol"], peer["ports"]["port"]]
    return allow, ports


class ConfigParser:
    def __init__(self, filepath=None):
        self.filepath = filepath
        self.containers = []
        self.policies = []

    def parse(self, filepath=None):
        if filepath is None:
            filepath = self.filepath
        if filepath is None:
            print("no filepath specified")
            return None

        if os.path.isfile(filepath):
            try:
                with open(filepath) as f:
                    self.create_object(load(f, Loader=Loader))
            except:  # noqa: E722  (bare except as in parser.py:32)
                print("Error opening or reading file " + filepath)
        else:
            try:
                for subdir, _dirs, files in os.walk(filepath):
                    for name in files:
                        with open(os.path.join(subdir, name)) as f:
                            self.create_object(load(f, Loader=Loader))
            except:  # noqa: E722  (bare except as in parser.py:46)
                print("Error opening or reading directory")
        return self.containers, self.policies

    def create_object(self, data):
        kind = data["kind"]
        if kind == "NetworkPolicy":
            spec = data["spec"]
            select = spec["podSelector"]["matchLabels"]
            name = data["metadata"]["name"]
            for ptype, rules_key, peers_key, suffix, direction in (
                    ("Ingress", "ingress", "from", "-ingress", PolicyIngress),
                    ("Egress", "egress", "to", "-egress", PolicyEgress)):
                if ptype not in spec["policyTypes"]:
                    continue
                for rule in spec[rules_key]:
                    allow, ports = _rule_allow(rule[peers_key])
                    self.policies.append(Policy(name + suffix, PolicySelect(select),
                                                PolicyAllow(allow), direction, ports))
        elif kind == "Pod":
            labels = data["metadata"]["labels"]
            for c in data["spec"]["containers"]:
                self.containers.append(Container(c["name"], labels))

    def print_all(self):
        for c in self.containers:
            print(c)
        for p in self.policies:
            print(p)


def main():
    cp = ConfigParser()
    cp.parse("data")
    cp.print_all()


if __name__ == "__main__":
    main()
